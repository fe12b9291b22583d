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

#define QA_DEVICE __device__ __forceinline__
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// ---------------------------------------------------------------- MFMA wrappers
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
// Round-to-nearest-even packs (gfx950 VOP3 v_cvt_pk_{f16,bf16}_f32).
QA_DEVICE unsigned pk_f16(float lo, float hi) {
  unsigned r;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}
QA_DEVICE unsigned pk_bf16(float lo, float hi) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
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
