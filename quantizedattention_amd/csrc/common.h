// Shared device helpers for the gfx950 (CDNA4) quantized-attention kernels.
//
// Everything here is CDNA4-only: wave64, MFMA 32x32 tiles, ds_read_b64_tr_b16, v_cvt_pk_*.
// MFMA fragment maps used throughout (cdna_hip_programming.md §3, verified by the
// mfma_layout_probe kernel and tests/test_gpu_layout.py):
//   32x32 C/D (every dtype):   lane l, reg r  ->  row (r&3) + 8*(r>>2) + 4*(l>>5), col l&31
//   f16/bf16 32x32x16 A/B:     lane l holds A[row l&31][k = 8*(l>>5) + j], j = 0..7
//   i8 32x32x32 A/B:           lane l holds A[row l&31][k = 16*(l>>5) + j], j = 0..15
// An accumulator X (rows in registers) used as the B operand of a following 32x32x16 product
// sums over X's rows in the permuted order  k(s, h, j) = 16s + 8(j>>2) + 4h + (j&3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "qattn.h"  // the C ABI: every extern "C" definition is checked against its declaration

namespace qattn {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef _Float16 v4h __attribute__((ext_vector_type(4)));
typedef _Float16 v2h __attribute__((ext_vector_type(2)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef int v2i __attribute__((ext_vector_type(2)));

#define QA_DEVICE __device__ __forceinline__
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// ---------------------------------------------------------------- host: dynamic-LDS grants
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) only when a launch needs more dynamic LDS than
// the kernel was granted so far: `granted` is a static of the calling launch function (one per
// kernel instantiation), so steady-state launches (decode steps of ~50 us) make no attribute call.
// The attribute belongs to the kernel on the CURRENT device, so the grant is kept per device (one
// process driving several GPUs must set it on each).
struct LdsGrant {
  static constexpr int MAX_DEV = 64;
  int bytes[MAX_DEV] = {};
};
inline bool lds_grant(const void* kernel, int bytes, LdsGrant& grants) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= LdsGrant::MAX_DEV) {
    (void)hipGetLastError();
    dev = -1;   // (unknown device: set the attribute, remember nothing)
  }
  int scratch = 0;
  int& granted = dev >= 0 ? grants.bytes[dev] : scratch;
  if (bytes <= granted) return true;
  if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
    // clear the runtime's last error: the caller reports the refusal (status 1), and a stale
    // hipErrorInvalidValue would otherwise surface in the host program's next unrelated HIP call
    (void)hipGetLastError();
    return false;
  }
  granted = bytes;
  return true;
}

// ---------------------------------------------------------------- MFMA wrappers
// f(std::integral_constant<int, 0>{}) .. f(std::integral_constant<int, N - 1>{}): a loop body
// instantiated per index, so ring slots and similar indices are compile-time constants in it
template <typename F, int... I>
QA_DEVICE void static_for_seq(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
QA_DEVICE void static_for(F&& f) {
  static_for_seq(f, std::make_integer_sequence<int, N>{});
}

QA_DEVICE v16i mfma_i8(v4i a, v4i b, v16i c) {
  return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}
QA_DEVICE v16f mfma_f16(v8h a, v8h b, v16f c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
QA_DEVICE v16f mfma_bf16(v8bf a, v8bf b, v16f c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- conversions
// Round-to-nearest-even packs (gfx950 v_cvt_pk_{f16,bf16}_f32, emitted by hipcc for these vector
// conversions).  Deliberately NOT inline asm: the results feed MFMA operands, and hipcc inserts the
// VALU-write -> MFMA-read wait states only for producers it can see.
typedef __bf16 v2bf_ __attribute__((ext_vector_type(2)));
typedef float v2f_ __attribute__((ext_vector_type(2)));
QA_DEVICE unsigned pk_f16(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((v2f_{lo, hi}), v2h));
}
QA_DEVICE unsigned pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((v2f_{lo, hi}), v2bf_));
}
QA_DEVICE float bf16_bits_to_f32(unsigned short b) { return __uint_as_float(((unsigned)b) << 16); }
// RNE f32 -> bf16 -> f32 (value rounding only).
QA_DEVICE float rne_bf16(float x) {
  unsigned u = __float_as_uint(x);
  if ((u & 0x7f800000u) == 0x7f800000u) return x;  // inf / nan pass through
  u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
  return __uint_as_float(u);
}
QA_DEVICE float rne_f16(float x) { return (float)(_Float16)x; }

QA_DEVICE float exp2_f32(float x) { return __builtin_amdgcn_exp2f(x); }
QA_DEVICE float log2_f32(float x) { return __builtin_amdgcn_logf(x); }

// ---------------------------------------------------------------- cross-lane
QA_DEVICE float xor32_f(float x) { return __shfl_xor(x, 32); }
QA_DEVICE float wave_max_f(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}

// Single-instruction max (hipcc otherwise canonicalises both fmaxf inputs with extra v_max).
QA_DEVICE float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// Full-wave max via DPP + permlane swaps (no LDS traffic); result in every lane.
QA_DEVICE float wave_max_dpp(float x) {
  x = vmax(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true)));
  x = vmax(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true)));
  x = vmax(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, true)));
  x = vmax(x, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, true)));
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
  auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax(__uint_as_float(r2[0]), __uint_as_float(r2[1]));
}
// Full-wave max of non-negative floats (no -0, no NaN), result in every lane: for such values the
// float order is the integer order of the bits, and the integer max lets hipcc fold each DPP move
// into its max (v_max_i32_dpp: one instruction per step, where the float form needs a move and a
// canonicalising max).  Bit-identical to wave_max_dpp on these inputs.
QA_DEVICE float wave_max_nonneg(float x) {
  int v = __float_as_int(x);
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true));    // quad_perm [1,0,3,2]
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true));    // quad_perm [2,3,0,1]
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));   // row_half_mirror
  v = max(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));   // row_mirror
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  v = max((int)r[0], (int)r[1]);
  const auto r2 = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  return __int_as_float(max((int)r2[0], (int)r2[1]));
}
// Two such maxima at once: the steps of the two chains interleave, so each DPP read of a value
// written one instruction earlier finds the other chain's step in between instead of an s_nop.
QA_DEVICE void wave_max2_nonneg(float& x, float& y) {
  int a = __float_as_int(x), b = __float_as_int(y);
  a = max(a, __builtin_amdgcn_mov_dpp(a, 0xB1, 0xF, 0xF, true));
  b = max(b, __builtin_amdgcn_mov_dpp(b, 0xB1, 0xF, 0xF, true));
  a = max(a, __builtin_amdgcn_mov_dpp(a, 0x4E, 0xF, 0xF, true));
  b = max(b, __builtin_amdgcn_mov_dpp(b, 0x4E, 0xF, 0xF, true));
  a = max(a, __builtin_amdgcn_mov_dpp(a, 0x141, 0xF, 0xF, true));
  b = max(b, __builtin_amdgcn_mov_dpp(b, 0x141, 0xF, 0xF, true));
  a = max(a, __builtin_amdgcn_mov_dpp(a, 0x140, 0xF, 0xF, true));
  b = max(b, __builtin_amdgcn_mov_dpp(b, 0x140, 0xF, 0xF, true));
  const auto ra = __builtin_amdgcn_permlane16_swap((unsigned)a, (unsigned)a, false, false);
  const auto rb = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
  a = max((int)ra[0], (int)ra[1]);
  b = max((int)rb[0], (int)rb[1]);
  const auto sa = __builtin_amdgcn_permlane32_swap((unsigned)a, (unsigned)a, false, false);
  const auto sb = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  x = __int_as_float(max((int)sa[0], (int)sa[1]));
  y = __int_as_float(max((int)sb[0], (int)sb[1]));
}
// Value of lane l^32 (half-wave exchange without LDS).  v_permlane32_swap vdst, vsrc swaps
// vdst[32..63] with vsrc[0..31]: with vdst = vsrc = x, lanes 0-31 find x[l+32] in the new vsrc and
// lanes 32-63 find x[l-32] in the new vdst.
QA_DEVICE unsigned xor32_swap_u(unsigned x, int lane) {
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return (lane < 32) ? r[1] : r[0];
}
QA_DEVICE float xor32_swap(float x, int lane) {
  return __uint_as_float(xor32_swap_u(__float_as_uint(x), lane));
}

// Sum / max over the lane pair (l, l^32), result in both lanes.
QA_DEVICE float pair_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
QA_DEVICE float pair_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Packed-half transcendental / rounding helpers on 4 pairs: low halves with the e32 form, then high
// halves with SDWA writing WORD_1 and preserving WORD_0 (hipcc would otherwise unpack, compute and
// v_pack_b32_f16).  The SDWA UNUSED_PRESERVE read of a VALU-written destination needs 2 wait
// states; the 3 independent instructions between each pair provide them (tests/test_gpu_layout.py).
#define QA_PK4(OP)                                                                              \
  asm(OP "_e32 %0, %4\n\t" OP "_e32 %1, %5\n\t" OP "_e32 %2, %6\n\t" OP "_e32 %3, %7\n\t"      \
      OP "_sdwa %0, %4 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"           \
      OP "_sdwa %1, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"           \
      OP "_sdwa %2, %6 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"           \
      OP "_sdwa %3, %7 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1"                 \
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])                                      \
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]))
QA_DEVICE void exp2_pk4(const v2h* x, v2h* r) { QA_PK4("v_exp_f16"); }
QA_DEVICE void trunc_pk4(const v2h* x, v2h* r) { QA_PK4("v_trunc_f16"); }

// ---------------------------------------------------------------- int8 block quantiser
// idx = trunc(RNE_f16(fp32(x) / s)) (int8:178-186: IEEE fp32 division, fp16 rounding, trunc) for
// fp16 x and the block scale s = f16(amax / 127), without a division per element: r = v_rcp_f32(s)
// (1 ulp), q0 = x r and one Newton step q1 = q0 + (x - q0 s) r, so |q1 - x/s| <= 0.5 ulp + 2^-44
// |x/s|.  x / s is never an fp16 rounding midpoint and lies at least one fp32 ulp away from every
// midpoint (a midpoint's odd 12-bit significand times the significand of s has more than the 11
// bits of x), so RNE_f16(q1) = RNE_f16(x / s) bit for bit -- checked exhaustively over every fp16
// x and s (qattn_probe_quant_div, tests/test_gpu_layout.py).  r = 0 for s = 0 gives q1 = 0 (the
// reference's idx 0 for an all-zero block).
QA_DEVICE float quant_rcp(float s) { return s != 0.f ? __builtin_amdgcn_rcpf(s) : 0.f; }
QA_DEVICE float quant_div(float x, float s, float r) {
  const float q0 = x * r;
  return __builtin_fmaf(__builtin_fmaf(-q0, s, x), r, q0);
}
// 8 fp16 values of a block -> their int8 indices (lo: values 0..3, hi: 4..7, byte j = index j)
// and the indices as exact floats (for the bf16 / f16 images).  trunc on packed halves, then
// y = t + 1536 (exact: the fp16 spacing is 1 in [1024, 2048)) holds t in its low byte and gives
// t = y - 1536 as a float without a -0.
QA_DEVICE void quant8(const v8h& x, float s, float r, unsigned& lo, unsigned& hi, float* qf) {
  v2h h[4], t[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    h[k] = __builtin_bit_cast(v2h, pk_f16(quant_div((float)x[2 * k], s, r),
                                          quant_div((float)x[2 * k + 1], s, r)));
  trunc_pk4(h, t);
  const v2h k1536 = {(_Float16)1536.0f, (_Float16)1536.0f};
  unsigned u[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const v2h y = t[k] + k1536;
    u[k] = __builtin_bit_cast(unsigned, y);
    qf[2 * k] = (float)y[0] - 1536.0f;
    qf[2 * k + 1] = (float)y[1] - 1536.0f;
  }
  lo = __builtin_amdgcn_perm(u[1], u[0], 0x06040200u);
  hi = __builtin_amdgcn_perm(u[3], u[2], 0x06040200u);
}

// d[j] = {f16(a[2j]*c + n), f16(a[2j+1]*c + n)}, one rounding each (v_fma_mix, f32 sources).  All 8
// low halves are written before the high halves so that no mixhi reads a just-written VGPR.
QA_DEVICE void fma_mix8(const float* a, float c, float n, v2h* d) {
  unsigned r[8];
  asm("v_fma_mixlo_f16 %0, %8, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %10, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %2, %12, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %3, %14, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %4, %16, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %5, %18, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %6, %20, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %7, %22, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %9, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %1, %11, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %2, %13, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %3, %15, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %4, %17, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %5, %19, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %6, %21, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %7, %23, %24, %25 op_sel_hi:[0,0,0]"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]),
        "=&v"(r[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
        "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(a[12]), "v"(a[13]), "v"(a[14]),
        "v"(a[15]), "v"(c), "v"(n));
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = __builtin_bit_cast(v2h, r[j]);
}
// f16(a*c) with one rounding (the same v_fma_mix rounding as fma_mix8, so that a row max computed
// from the int32 maximum equals the max of the fma_mix8 results bit for bit)
QA_DEVICE _Float16 mul_mix(float a, float c) {
  unsigned r;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0 op_sel_hi:[0,0,0]" : "=v"(r) : "v"(a), "v"(c));
  return __builtin_bit_cast(v2h, r)[0];
}
// f16(a*c + n), one rounding
QA_DEVICE _Float16 fma_mix1(float a, float c, float n) {
  unsigned r;
  asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[0,0,0]" : "=v"(r) : "v"(a), "v"(c), "v"(n));
  return __builtin_bit_cast(v2h, r)[0];
}

// ---------------------------------------------------------------- biased int32 accumulators
// An int8 MFMA started from C = KMAG_BITS instead of 0 adds the exact integer dot X to the bit
// pattern of the fp32 value 1.5 * 2^23, whose spacing is 1: read as fp32 the accumulator is exactly
// KMAG + X for |X| < 2^22 (a 32x32x32 i8 dot is at most 32 * 128 * 128 * (D/32) < 2^22 for D <= 128).
// The int -> float conversion disappears: f(acc) * c - KMAG * c is X * c in one fused operation, and
// KMAG * c is exact when c has at most 23 significant bits (kmag_scale clears the last one).  The
// biased values still order like X as signed int32 (a row max can run on the raw accumulator).
constexpr int KMAG_BITS = 0x4B400000;
constexpr float KMAG = 12582912.0f;   // 1.5 * 2^23
QA_DEVICE float kmag_scale(float c) { return __uint_as_float(__float_as_uint(c) & ~1u); }

// d[j] = {f16(a[2j]*c + n), f16(a[2j+1]*c + n)} for the 16 values of a biased accumulator (the same
// v_fma_mix rounding as fma_mix8).  `dep` must be a value the compiler computed FROM those
// accumulator registers (e.g. their row max): hipcc inserts the MFMA-result -> VALU wait states only
// for its own instructions, so this asm has to be ordered after one of them; the operand makes it so.
QA_DEVICE void fma_mix16_after(const v16i& acc, float c, float n, int dep, v2h* d) {
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = __int_as_float(acc[i]);
  unsigned r[8];
  asm("v_fma_mixlo_f16 %0, %8, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %10, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %2, %12, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %3, %14, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %4, %16, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %5, %18, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %6, %20, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %7, %22, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %9, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %1, %11, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %2, %13, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %3, %15, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %4, %17, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %5, %19, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %6, %21, %24, %25 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %7, %23, %24, %25 op_sel_hi:[0,0,0]"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]),
        "=&v"(r[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
        "v"(a[8]), "v"(a[9]), "v"(a[10]), "v"(a[11]), "v"(a[12]), "v"(a[13]), "v"(a[14]),
        "v"(a[15]), "v"(c), "v"(n), "v"(dep));
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = __builtin_bit_cast(v2h, r[j]);
}
// The same S = f16(X c) from a biased accumulator through f32: one v_pk_fma_f32 per pair (the
// exact (KMAG + X) c - KMAG c, rounded to f32) and one v_cvt_pk_f16_f32 (RNE).  Two roundings (f32,
// then f16) where fma_mix16_after has one: the f16 results differ only where f32(X c) lands on an
// f16 rounding midpoint.  Issue cost ~12.9 cycles per pair against ~16.7 for two v_fma_mix{lo,hi}
// (tools/ubench/coexec2.py: v_fma_mix*_f16 issue like transcendentals, ~8.4 cycles).  Compiler
// builtins, so hipcc inserts the MFMA-result -> VALU wait states itself.
QA_DEVICE void biased_to_f16x16(const v16i& acc, float c, float nb, v2h* d) {
  const v2f_ c2 = {c, c}, n2 = {nb, nb};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const v2f_ a = {__int_as_float(acc[2 * j]), __int_as_float(acc[2 * j + 1])};
    d[j] = __builtin_convertvector(__builtin_elementwise_fma(a, c2, n2), v2h);
  }
}
QA_DEVICE _Float16 biased_to_f16(int a, float c, float nb) {
  return (_Float16)__builtin_fmaf(__int_as_float(a), c, nb);
}

// f32(x.lo) + f32(x.hi) of a packed f16 pair in one v_fma_mix_f32
QA_DEVICE float pk_hsum(v2h x) {
  float r;
  asm("v_fma_mix_f32 %0, %1, 1.0, %1 op_sel:[0,0,1] op_sel_hi:[1,0,1]"
      : "=v"(r) : "v"(__builtin_bit_cast(unsigned, x)));
  return r;
}
// y = RTZ_f16(w * e + 1024) = 1024 + trunc(w * e) for 0 <= w * e < 1024 (the f16 spacing is 1 in
// [1024, 2048)): byte 0 / byte 2 of y are the int8 indices trunc(w * e) of the two halves.
// MODE.FP_ROUND[3:2] (f16/f64) = 3 (toward zero) only around the 8 ops.
QA_DEVICE void p_index8(const v2h* e, v2h w2, unsigned* y) {
  const v2h k1024 = {(_Float16)1024.0f, (_Float16)1024.0f};
  asm("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3\n\t"
      "s_nop 1\n\t"
      "v_pk_fma_f16 %0, %8, %16, %17\n\t"
      "v_pk_fma_f16 %1, %9, %16, %17\n\t"
      "v_pk_fma_f16 %2, %10, %16, %17\n\t"
      "v_pk_fma_f16 %3, %11, %16, %17\n\t"
      "v_pk_fma_f16 %4, %12, %16, %17\n\t"
      "v_pk_fma_f16 %5, %13, %16, %17\n\t"
      "v_pk_fma_f16 %6, %14, %16, %17\n\t"
      "v_pk_fma_f16 %7, %15, %16, %17\n\t"
      "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 0\n\t"
      "s_nop 1"
      : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "=&v"(y[4]), "=&v"(y[5]), "=&v"(y[6]),
        "=&v"(y[7])
      : "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(e[3]), "v"(e[4]), "v"(e[5]), "v"(e[6]), "v"(e[7]),
        "v"(w2), "v"(k1024));
}
// Pack the int8 indices of p_index8 into the i8 MFMA operand: byte j = index j (j = 0..15), i.e.
// byte 0 of y[j/2] half j%2.
QA_DEVICE v4i pack_p_index(const unsigned* y) {
  v4i r;
#pragma unroll
  for (int w = 0; w < 4; ++w) r[w] = (int)__builtin_amdgcn_perm(y[2 * w + 1], y[2 * w], 0x06040200u);
  return r;
}
// The low bytes of the 16 int32 values of an accumulator, packed in register order (byte j of the
// result = low byte of t[j]): the i8 operand of a following MFMA.
QA_DEVICE v4i pack_acc_bytes(const v16i& t) {
  v4i r;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const unsigned lo = __builtin_amdgcn_perm((unsigned)t[4 * w + 1], (unsigned)t[4 * w], 0x0c0c0400u);
    const unsigned hi = __builtin_amdgcn_perm((unsigned)t[4 * w + 3], (unsigned)t[4 * w + 2], 0x0c0c0400u);
    r[w] = (int)__builtin_amdgcn_perm(hi, lo, 0x05040100u);
  }
  return r;
}
// B operand of the 32x32 identity for v_mfma_i32_32x32x32_i8: lane l holds B[k = 16h + j][l & 31],
// byte j = (16h + j == l & 31).  X . I with X as the A operand (lane = row, 16 consecutive k bytes)
// returns X in the accumulator layout (lane = column, rows in registers): a register transpose.
QA_DEVICE v4i identity_b_i8(int lane) {
  const int j = (lane & 31) - 16 * (lane >> 5);
  v4i r = {0, 0, 0, 0};
  if (j >= 0 && j < 16) r[j >> 2] = 1 << (8 * (j & 3));
  return r;
}
// y = RTZ_f16(127 e + 1024) = P_i8 + 1024 (exact integer), then w = RNE_f16(y*sp - 1024*sp) =
// f16(P_i8 * sp).  MODE.FP_ROUND[3:2] (f16/f64) = 3 (toward zero) only around the first 8 ops.
QA_DEVICE void p_operand8(const v2h* e, v2h sp2, v2h nsp2, v2h* w) {
  const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
  const v2h k1024 = {(_Float16)1024.0f, (_Float16)1024.0f};
  v2h y[8];
  asm volatile(
      "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3\n\t"
      "s_nop 1\n\t"
      "v_pk_fma_f16 %0, %8, %16, %17\n\t"
      "v_pk_fma_f16 %1, %9, %16, %17\n\t"
      "v_pk_fma_f16 %2, %10, %16, %17\n\t"
      "v_pk_fma_f16 %3, %11, %16, %17\n\t"
      "v_pk_fma_f16 %4, %12, %16, %17\n\t"
      "v_pk_fma_f16 %5, %13, %16, %17\n\t"
      "v_pk_fma_f16 %6, %14, %16, %17\n\t"
      "v_pk_fma_f16 %7, %15, %16, %17\n\t"
      "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 0\n\t"
      "s_nop 1"
      : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3]), "=&v"(y[4]), "=&v"(y[5]), "=&v"(y[6]),
        "=&v"(y[7])
      : "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(e[3]), "v"(e[4]), "v"(e[5]), "v"(e[6]), "v"(e[7]),
        "v"(k127), "v"(k1024));
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = __builtin_elementwise_fma(y[j], sp2, nsp2);
}

// LDS-DMA of one 16-B chunk per lane: the LDS destination is lds_base (wave-uniform) + 16*lane.
// Issued from inline asm on purpose: hipcc cannot tell which LDS bytes a global_load_lds writes, so
// for the builtin form it inserts s_waitcnt vmcnt(0) before every later ds_read (serialising the
// prefetch of block j+1 with the compute of block j).  The asm form is invisible to its waitcnt
// pass; the kernel waits for its own DMAs with dma_wait() before the barrier that publishes them.
QA_DEVICE void glds16(const void* gsrc, void* lds_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(lds_base));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}
// LDS-DMA with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset (global SADDR
// form): no per-lane 64-bit address arithmetic in the loop.
QA_DEVICE void glds16_s(const void* sbase, unsigned voff, void* lds_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(lds_base));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}
// dword LDS-DMA (64 lanes x 4 B = 256 B, lane-linear destination), SADDR form
QA_DEVICE void glds4_s(const void* sbase, unsigned voff, void* lds_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(lds_base));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}
// LDS-ring step: wait until at most N of this wave's VMEM ops (the LDS-DMA of later tiles) are in
// flight and all its LDS reads returned, then workgroup barrier (publishes the landed tile and
// frees the oldest slot).
// (-DQA_RING_DRAIN=1, diagnostic builds: wait for every VMEM op instead -- no DMA in flight across a
// barrier, which rules the ring's wait counts out as the cause of a result)
#ifndef QA_RING_DRAIN
#define QA_RING_DRAIN 0
#endif
template <int N>
QA_DEVICE void ring_wait_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(QA_RING_DRAIN ? 0 : N) : "memory");
}
// ---------------------------------------------------------------- buffer LDS-DMA (ring staging)
// buffer_load_dword{x4} ... offen lds: source = V#.base + voffset (lane-constant, swizzle applied)
// + soffset (wave-uniform tile offset, SGPR); LDS destination = M0 + 16*lane (4*lane for dword).
// Per piece only the M0 write and the load issue: no 64-bit per-lane address arithmetic.  M0 is
// written without save/restore: the kernels that use these helpers contain no other M0 use
// (tests/test_isa.py proves on the emitted code that hipcc itself never reads or writes M0 and that every
// LDS-DMA follows an M0 write in its own asm block), and the M0 -> LDS-DMA hazard takes one s_nop.
QA_DEVICE v4u make_rsrc(const void* base, unsigned bytes) {
  const unsigned long a = (unsigned long)base;
  v4u r;
  r[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32) & 0xffffu);   // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(bytes);                            // range checked
  r[3] = 0x00020000u;
  return r;
}
QA_DEVICE unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)(p));
}
QA_DEVICE void dma16_buf(v4u rsrc, unsigned voff, unsigned soff, unsigned lds) {
  soff = __builtin_amdgcn_readfirstlane(soff);   // wave-uniform by construction; keep them in SGPRs
  lds = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               ::"v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}
// The same with the non-temporal policy, for bytes read exactly once (MI355X_MICROARCH "nt-weights":
// issue -> landed ~18 % shorter on once-read streams).
QA_DEVICE void dma16_buf_nt(v4u rsrc, unsigned voff, unsigned soff, unsigned lds) {
  soff = __builtin_amdgcn_readfirstlane(soff);
  lds = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen nt lds"
               ::"v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}
QA_DEVICE void dma4_buf(v4u rsrc, unsigned voff, unsigned soff, unsigned lds) {
  soff = __builtin_amdgcn_readfirstlane(soff);
  lds = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %0, %1, %2 offen lds"
               ::"v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
               : "memory");
}

// s_waitcnt vmcnt(0) as a real instruction hipcc's waitcnt pass understands: retire every ordinary
// global load before a loop that issues asm LDS-DMA (otherwise the compiler's first-use wait for
// those loads lands inside the loop and also waits for the in-flight DMA).
QA_DEVICE void vmem_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// Wait for every outstanding VMEM op of this wave (e.g. LDS-DMA still landing before the wave exits).
QA_DEVICE void vmcnt_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Wait for every outstanding VMEM op of this wave (incl. LDS-DMA) and LDS op, then barrier.
QA_DEVICE void dma_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, cols 4p..4p+3 of a 4x16
// block; lane i receives column i of the 4 rows (cdna_hip_programming.md T10).
QA_DEVICE v4s ds_read_tr16(const void* lds_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4s*)(const_cast<void*>(lds_addr)));
}

// Two transposed reads concatenated into one 8 x 16-bit MFMA operand.  Build the vector with
// __builtin_shufflevector only: assembling it element-wise from the v4i16 results miscompiles on
// ROCm 7.2 (the backend splats element 0; seen in the .s as v_perm_b32 vX, vX, vX, 0x5040100).
QA_DEVICE v8s ds_read_tr16_x2(const void* addr0, const void* addr1) {
  const v4s a0 = ds_read_tr16(addr0);
  const v4s a1 = ds_read_tr16(addr1);
  return __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
}

// ---------------------------------------------------------------- row-major tile stores
// A wave's 32-row x D output tile in the transposed 32x32 MFMA layout (acc[b][r] holds element
// d = 32b + 8(r>>2) + 4h + (r&3) of row l&31) written as whole rows: staged through the wave's own
// LDS region (row pitch padded by 16 B: the 8-/16-B per-row writes are bank-conflict-free), then
// read back 16 B per lane and stored with fully coalesced 16-B global stores (a 1-KiB span per
// instruction).  Storing straight from the MFMA layout touches 32 rows per instruction with 8-16 B
// each, which made the epilogue dominate short kernels.
// NPASS > 1 stages D / NPASS columns at a time through a proportionally smaller region (kernels
// whose LDS budget is set by the ring, not by the epilogue).
template <int D, typename T, int NPASS = 1>
struct RowTile {
  static constexpr int DC = D / NPASS;                      // columns per pass
  static constexpr int PITCH = DC * (int)sizeof(T) + 16;
  static constexpr int BYTES = 32 * PITCH;
};
// Element value written: acc * sc, or fma(acc, sc, add) when AFFINE.
template <int D, typename T, int NPASS = 1, bool AFFINE = false>
QA_DEVICE void store_rows(const v16f* acc, float sc, char* lds, T* dst_row0, int lane,
                          float add = 0.f) {
  using RT = RowTile<D, T, NPASS>;
  constexpr int NBP = D / 32 / NPASS;                        // 32-wide d blocks per pass
  const int h = lane >> 5, c32 = lane & 31;
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
#pragma unroll
    for (int bb = 0; bb < NBP; ++bb) {
      const int b = pass * NBP + bb;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        char* p = lds + c32 * RT::PITCH + (32 * bb + 8 * g + 4 * h) * (int)sizeof(T);
        if constexpr (sizeof(T) == 2) {
          v4h w;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            w[j] = (_Float16)(AFFINE ? fmaf(acc[b][4 * g + j], sc, add) : acc[b][4 * g + j] * sc);
          *reinterpret_cast<v4h*>(p) = w;
        } else {
          v4f w;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            w[j] = AFFINE ? fmaf(acc[b][4 * g + j], sc, add) : acc[b][4 * g + j] * sc;
          *reinterpret_cast<v4f*>(p) = w;
        }
      }
    }
    constexpr int CPR = RT::DC * (int)sizeof(T) / 16;   // 16-B chunks per staged row
    constexpr int RPI = 64 / CPR;                       // rows per instruction
    const int r = lane / CPR, c = lane % CPR;
#pragma unroll
    for (int i = 0; i < 32 / RPI; ++i) {
      const int row = i * RPI + r;
      const v4u v = *reinterpret_cast<const v4u*>(lds + row * RT::PITCH + 16 * c);
      *reinterpret_cast<v4u*>(reinterpret_cast<char*>(dst_row0) + (long)row * D * (long)sizeof(T) +
                              pass * RT::DC * (int)sizeof(T) + 16 * c) = v;
    }
  }
}

// Causal grids: the work of a workgroup grows with its query block (forward, dQ) or shrinks with
// its key block (dK/dV).  Dispatch the heaviest block of every head first -- longest-processing-
// time order, so the light blocks fill the tail -- with every head still on XCD bh & 7.
// heavy_last: the heaviest block is the last index (query blocks), else the first (key blocks).
// Speed only, never correctness.
QA_DEVICE void xcd_remap_lpt(int bid, int nq, int nbh, bool heavy_last, int& bh, int& qt) {
  int r;
  if ((nbh & 7) == 0) {
    const int hpx = nbh >> 3, j = bid >> 3;
    r = j / hpx;
    bh = (j % hpx) * 8 + (bid & 7);
  } else {
    r = bid / nbh;
    bh = bid % nbh;
  }
  qt = heavy_last ? nq - 1 - r : r;
}

// xcd_remap_lpt over groups of hg heads per XCD: the groups run one after another, longest-first
// inside a group.  Fewer heads in flight per XCD (hg instead of nbh / 8) keep the blocks of one head
// that stream the same rows close together in time, for L2 reuse.  hg must divide nbh / 8.
QA_DEVICE void xcd_remap_lpt_grouped(int bid, int nq, int nbh, bool heavy_last, int hg, int& bh, int& qt) {
  if ((nbh & 7) != 0 || ((nbh >> 3) % hg) != 0) {
    xcd_remap_lpt(bid, nq, nbh, heavy_last, bh, qt);
    return;
  }
  const int xcd = bid & 7, j = bid >> 3;
  const int g = j / (hg * nq), k = j % (hg * nq);
  const int r = k / hg;
  bh = (g * hg + k % hg) * 8 + xcd;
  qt = heavy_last ? nq - 1 - r : r;
}

// Workgroup -> (head, q-tile) remap that keeps every q-tile of one head on one XCD
// (blocks b and b+8 share an XCD under round-robin dispatch; speed only, never correctness).
QA_DEVICE void xcd_remap(int bid, int nq, int nbh, int& bh, int& qt) {
  const int total = nq * nbh;
  if ((nbh & 7) == 0) {
    const int xcd = bid & 7, j = bid >> 3;
    qt = j % nq;
    bh = (j / nq) * 8 + xcd;
  } else {
    bh = bid / nq;
    qt = bid % nq;
  }
  (void)total;
}

}  // namespace qattn
