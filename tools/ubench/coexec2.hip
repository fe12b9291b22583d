// Role-split co-execution by instruction type (dev tool, tools/ubench/coexec2.py).  ONE workgroup
// per CU (96 KiB LDS), W waves per SIMD: waves 0..3 (one per SIMD) loop over 12 int8 MFMAs (4
// accumulator chains), the others over 144 vector instructions of ONE type (16 independent
// registers, inline asm, so the instruction is exactly the one named).  Per wave: cycles per
// iteration (s_memtime).  Question answered: which vector instruction types slow a co-resident
// MFMA-only wave down (share its pipe), and at what issue cost they run beside it.
#include <hip/hip_runtime.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__device__ __forceinline__ void valu16(unsigned* r, unsigned long* d, unsigned k, unsigned long kk) {
#define ONE(i)                                                                                  \
  if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r[i]) : "v"(k));        \
  if constexpr (OP == 1) asm volatile("v_pk_fma_f16 %0, %0, %1, %1" : "+v"(r[i]) : "v"(k));     \
  if constexpr (OP == 2) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(r[i]) : "v"(k));         \
  if constexpr (OP == 3) asm volatile("v_pk_max_f16 %0, %0, %1" : "+v"(r[i]) : "v"(k));         \
  if constexpr (OP == 4) asm volatile("v_exp_f16 %0, %0" : "+v"(r[i]));                          \
  if constexpr (OP == 5) asm volatile("v_exp_f32 %0, %0" : "+v"(r[i]));                          \
  if constexpr (OP == 6) asm volatile("v_fma_mixlo_f16 %0, %0, %1, %1 op_sel_hi:[0,0,0]" : "+v"(r[i]) : "v"(k)); \
  if constexpr (OP == 7) asm volatile("v_add_f16 %0, %0, %1" : "+v"(r[i]) : "v"(k));            \
  if constexpr (OP == 8) asm volatile("v_max_i32 %0, %0, %1" : "+v"(r[i]) : "v"(k));            \
  if constexpr (OP == 9) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(r[i]));                      \
  if constexpr (OP == 10) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r[i]) : "v"(k));      \
  if constexpr (OP == 11) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d[i]) : "v"(kk));   \
  if constexpr (OP == 12) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(d[i]) : "v"(kk));       \
  if constexpr (OP == 13) asm volatile("v_cvt_pk_f16_f32 %0, %1, %1" : "=v"(r[i]) : "v"(r[i]));   \
  if constexpr (OP == 14) asm volatile("v_fma_mix_f32 %0, %0, %1, %1 op_sel_hi:[0,0,0]" : "+v"(r[i]) : "v"(k)); \
  if constexpr (OP == 15) asm volatile("v_cvt_f16_f32 %0, %0" : "+v"(r[i]));                       \
  if constexpr (OP == 16) asm volatile("v_pk_mul_f16 %0, %0, %1" : "+v"(r[i]) : "v"(k));          \
  if constexpr (OP == 17) asm volatile("v_max3_i32 %0, %0, %1, %1" : "+v"(r[i]) : "v"(k));        \
  if constexpr (OP == 18) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(r[i]) : "v"(k));            \
  if constexpr (OP == 19) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r[i]) : "v"(k));
  R16(ONE)
#undef ONE
}

// MIX: waves 0..3 interleave their 12 MFMAs with the 144 vector instructions (one mixed wave per
// SIMD, the others idle), the mixed-kernel pattern
template <int OP, bool MIX>
__global__ __launch_bounds__(1024) void coexec2_kernel(long long* out, int iters, int m_iters) {
  extern __shared__ char lds[];
  unsigned r[16];
  unsigned long d[16];
  for (int i = 0; i < 16; ++i) r[i] = 0x3c003c00u + threadIdx.x + i;
  for (int i = 0; i < 16; ++i) d[i] = 0x3f8000003f800000ul + threadIdx.x + i;
  const unsigned k = 0x3c003c01u;
  const unsigned long kk = 0x3f8000013f800001ul;
  v4i a = {1 + (int)threadIdx.x, 2, 3, (int)threadIdx.x};
  v16i c[4];
  for (int j = 0; j < 4; ++j) c[j] = v16i{};
  const int wave = threadIdx.x >> 6;
  lds[threadIdx.x] = 0;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  if (MIX) {
    if (wave < 4) {
      for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < 12; ++m) {
          c[m & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c[m & 3], 0, 0, 0);
          if (m % 4 == 3) { valu16<OP>(r, d, k, kk); valu16<OP>(r, d, k, kk); valu16<OP>(r, d, k, kk); }
        }
      }
    }
  } else if (wave < 4) {
    for (int it = 0; it < m_iters; ++it) {
#pragma unroll
      for (int m = 0; m < 12; ++m) c[m & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c[m & 3], 0, 0, 0);
    }
  } else {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int v = 0; v < 9; ++v) valu16<OP>(r, d, k, kk);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = lds[(threadIdx.x + 1) & 1023];
  for (int i = 0; i < 16; ++i) s += r[i] + (unsigned)d[i];
  for (int j = 0; j < 4; ++j) s += (unsigned)c[j][0];
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x >> 6) + wave;
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = (long long)s;
  }
}

// m_iters: iterations of the MFMA waves (0: they idle, the vector waves run alone; < 0: MIX)
extern "C" int coexec2(int op, int waves_per_simd, int iters, int m_iters, long long* out, int nblocks) {
  dim3 grid(nblocks), block(64 * 4 * waves_per_simd);
  const int lds = 96 * 1024;
#define K(N)                                                                                     \
  case N:                                                                                        \
    hipFuncSetAttribute((const void*)coexec2_kernel<N, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
    hipFuncSetAttribute((const void*)coexec2_kernel<N, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
    if (m_iters < 0) hipLaunchKernelGGL((coexec2_kernel<N, true>), grid, block, lds, 0, out, iters, 0);    \
    else hipLaunchKernelGGL((coexec2_kernel<N, false>), grid, block, lds, 0, out, iters, m_iters);         \
    break;
  switch (op) { K(0) K(1) K(2) K(3) K(4) K(5) K(6) K(7) K(8) K(9) K(10) K(11) K(12) K(13) K(14) K(15) K(16) K(17) K(18) K(19) }
#undef K
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
