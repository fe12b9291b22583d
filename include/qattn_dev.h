/*
 * qattn_dev.h — C ABI of libqattn_dev.so, the development library of fragment-layout probes.
 *
 * Not product API: these one-wave kernels check the lane maps and packed-math helpers that the
 * product kernels (libqattn.so, include/qattn.h) assume, on asymmetric integer data
 * (tests/test_gpu_layout.py, tools/probe_fp4.py).  Same conventions as qattn.h.
 */
#ifndef QATTN_DEV_H
#define QATTN_DEV_H

#ifdef __cplusplus
extern "C" {
#endif

/* MFMA / LDS-transpose fragment-layout probes (one wave). */
int qattn_probe_mfma_i8(const void* A, const void* B, void* C, void* stream);
int qattn_probe_mfma_f16(const void* A, const void* B, void* C, void* stream);
int qattn_probe_tr16(const void* M, void* out, void* stream);
int qattn_probe_pk(const void* x, void* e, void* t, void* stream);
/* int8-forward softmax helpers on 16 lanes: w = f16(trunc(127 e) * sp) via the round-toward-zero
 * packed fma; d = {f16(a*c + n)} via v_fma_mix (cn holds (c, n) per lane). */
int qattn_probe_fwd_helpers(const void* e, const void* sp, void* w, const void* a, const void* cn,
                            void* d, void* stream);

/* MX-FP4 probes: one block-scaled 32x32x64 fp4 MFMA (A, B: 64 lanes x 16 B of e2m1
 * nibbles, sa / sb: one e8m0 byte per lane, C: 64 x 16 f32) and the scaled fp4 pack/unpack converts
 * (lane i packs x[8i..8i+7] with scale s[i]). */
int qattn_probe_mfma_fp4(const void* A, const void* B, const void* sa, const void* sb, void* C,
                         void* stream);
int qattn_probe_fp4_cvt(const void* x, const void* s, void* packed, void* back, void* stream);

/* The int8 quantiser's division-free index (common.h quant8) vs the IEEE fp32 division, over every
 * finite fp16 x with |x| < 127.5 s (a block holds |x / s| <= 127.07) and the fp16 scales s with
 * bit patterns in [s_lo, s_hi); bad[0]
 * (unsigned[6], zeroed by the caller) counts mismatching indices / images, bad[1..5] = the first
 * (s bits, x bits, reference index, index, image bits). */
int qattn_probe_quant_div(int s_lo, int s_hi, void* bad, void* stream);

/* Device copy of `bytes` (a multiple of 16) by exactly `workgroups` workgroups of 256 threads
 * (grid-stride): an RCCL-like few-workgroup copy for the overlap probe (tools/overlap_probe.py). */
int qattn_probe_few_wg_copy(const void* src, void* dst, long bytes, int workgroups, void* stream);

/* exp2 on every fp16 argument h (65536 bit patterns): e32[h] = bits of v_exp_f32((float)h) (uint32),
 * e16[h] = bits of v_exp_f16(h) (uint16) -- tools/exp2_probe.py, tests/test_gpu_layout.py. */
int qattn_probe_exp2_dom(void* e32, void* e16, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* QATTN_DEV_H */
