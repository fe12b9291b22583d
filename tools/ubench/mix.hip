// Mixed-wave issue model (dev tool, tools/ubench/mix.py).  ONE workgroup per CU (96 KiB LDS), W
// waves per SIMD, EVERY wave runs the same loop: 8 MFMAs of one shape (4 independent accumulator
// chains) with P vector instructions of one type after each MFMA (16 registers round-robin, inline
// asm, so the instruction is exactly the one named).  Per wave: cycles per iteration (s_memtime).
// Question answered: per SIMD, how many cycles does a tile-wave of N MFMAs + V vector instructions
// of a given type take at 1..4 waves per SIMD -- the cost model of the int8 forward's loop.
#include <hip/hip_runtime.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v4i_ __attribute__((ext_vector_type(4)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int OP>
__device__ __forceinline__ void one(unsigned& r, unsigned long& d, unsigned k, unsigned long kk) {
  if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
  if constexpr (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(d) : "v"(kk));
  if constexpr (OP == 2) asm volatile("v_pk_fma_f16 %0, %0, %1, %1" : "+v"(r) : "v"(k));
  if constexpr (OP == 3) asm volatile("v_exp_f16 %0, %0" : "+v"(r));
  if constexpr (OP == 4) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(r) : "v"(k));
  if constexpr (OP == 5) asm volatile("v_cvt_pk_f16_f32 %0, %1, %1" : "=v"(r) : "v"(r));
  if constexpr (OP == 6) asm volatile("v_max3_i32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
  if constexpr (OP == 7) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r) : "v"(k));
  if constexpr (OP == 8) asm volatile("v_exp_f32 %0, %0" : "+v"(r));
  if constexpr (OP == 9) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(d) : "v"(kk));
  if constexpr (OP == 10) asm volatile("v_fma_mix_f32 %0, %0, %1, %1 op_sel_hi:[0,0,0]" : "+v"(r) : "v"(k));
  if constexpr (OP == 11) asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(k));
  if constexpr (OP == 12) asm volatile("v_fma_mixlo_f16 %0, %0, %1, %1 op_sel_hi:[0,0,0]" : "+v"(r) : "v"(k));
  if constexpr (OP == 13) asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(r));
  if constexpr (OP == 14) asm volatile("ds_read_b64 %0, %1" : "=v"(d) : "v"(k & 0xff8u));
  if constexpr (OP == 15) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(k));
  if constexpr (OP == 16) asm volatile("s_nop 0" ::);
}

// SHAPE 0: v_mfma_i32_32x32x32_i8, 1: v_mfma_i32_16x16x64_i8, 2: v_mfma_f32_32x32x16_f16,
//       3: v_mfma_f32_16x16x32_f16
template <int OP, int P, int SHAPE>
__global__ __launch_bounds__(1024) void mix_kernel(long long* out, int iters) {
  extern __shared__ char lds[];
  unsigned r[16];
  unsigned long d[16];
  for (int i = 0; i < 16; ++i) r[i] = 0x3c003c00u + threadIdx.x + i;
  for (int i = 0; i < 16; ++i) d[i] = 0x3f8000003f800000ul + threadIdx.x + i;
  const unsigned k = 0x3c003c01u;
  const unsigned long kk = 0x3f8000013f800001ul;
  v4i a = {1 + (int)threadIdx.x, 2, 3, (int)threadIdx.x};
  v8h ah = {(_Float16)1, (_Float16)2, (_Float16)0, (_Float16)1, (_Float16)1, (_Float16)2,
            (_Float16)0, (_Float16)1};
  v16i c[4];
  v4i c16[4];
  v16f cf[4];
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f cf16[4];
  for (int j = 0; j < 4; ++j) { c[j] = v16i{}; c16[j] = v4i{}; cf[j] = v16f{}; cf16[j] = v4f{}; }
  const int wave = threadIdx.x >> 6;
  lds[threadIdx.x] = 0;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  int ri = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if constexpr (SHAPE == 0) c[m & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c[m & 3], 0, 0, 0);
      if constexpr (SHAPE == 1) c16[m & 3] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c16[m & 3], 0, 0, 0);
      if constexpr (SHAPE == 2) cf[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ah, cf[m & 3], 0, 0, 0);
      if constexpr (SHAPE == 3) cf16[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, ah, cf16[m & 3], 0, 0, 0);
#pragma unroll
      for (int p = 0; p < P; ++p) one<OP>(r[(m * P + p) & 15], d[(m * P + p) & 15], k, kk);
      if constexpr (OP == 14) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  (void)ri;
  long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = lds[(threadIdx.x + 1) & 1023];
  for (int i = 0; i < 16; ++i) s += r[i] + (unsigned)d[i];
  for (int j = 0; j < 4; ++j) s += (unsigned)c[j][0] + (unsigned)c16[j][0] + (unsigned)cf[j][0] + (unsigned)cf16[j][0];
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x >> 6) + wave;
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = (long long)s;
  }
}

#define NP 6
static const int PVALS[NP] = {0, 4, 8, 12, 16, 24};

template <int OP, int SHAPE, int PI>
static void launch(dim3 grid, dim3 block, int lds, long long* out, int iters) {
  constexpr int P = PI == 0 ? 0 : PI == 1 ? 4 : PI == 2 ? 8 : PI == 3 ? 12 : PI == 4 ? 16 : 24;
  hipFuncSetAttribute((const void*)mix_kernel<OP, P, SHAPE>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL((mix_kernel<OP, P, SHAPE>), grid, block, lds, 0, out, iters);
}
template <int OP, int SHAPE>
static void launch_p(int pi, dim3 grid, dim3 block, int lds, long long* out, int iters) {
  switch (pi) {
    case 0: launch<OP, SHAPE, 0>(grid, block, lds, out, iters); break;
    case 1: launch<OP, SHAPE, 1>(grid, block, lds, out, iters); break;
    case 2: launch<OP, SHAPE, 2>(grid, block, lds, out, iters); break;
    case 3: launch<OP, SHAPE, 3>(grid, block, lds, out, iters); break;
    case 4: launch<OP, SHAPE, 4>(grid, block, lds, out, iters); break;
    default: launch<OP, SHAPE, 5>(grid, block, lds, out, iters); break;
  }
}
template <int OP>
static void launch_s(int shape, int pi, dim3 grid, dim3 block, int lds, long long* out, int iters) {
  switch (shape) {
    case 0: launch_p<OP, 0>(pi, grid, block, lds, out, iters); break;
    case 1: launch_p<OP, 1>(pi, grid, block, lds, out, iters); break;
    case 2: launch_p<OP, 2>(pi, grid, block, lds, out, iters); break;
    default: launch_p<OP, 3>(pi, grid, block, lds, out, iters); break;
  }
}

extern "C" int mix(int op, int shape, int pi, int waves_per_simd, int iters, long long* out, int nblocks) {
  dim3 grid(nblocks), block(64 * 4 * waves_per_simd);
  const int lds = 96 * 1024;
#define K(N) case N: launch_s<N>(shape, pi, grid, block, lds, out, iters); break;
  switch (op) { K(0) K(1) K(2) K(3) K(4) K(5) K(6) K(7) K(8) K(9) K(10) K(11) K(12) K(13) K(14) K(15) K(16) }
#undef K
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
