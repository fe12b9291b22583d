// Instruction-issue microbenchmarks for gfx950 (dev tool, not part of libqattn).
// Each wave runs ITER iterations of a block of 16 independent instructions of one kind on 16
// registers and records s_memtime cycles; a launch places W waves on every SIMD (grid = 256 CUs x
// 4 SIMDs x W waves) so the per-SIMD cost with 1 and 2 co-resident waves can be compared.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define REP16(X) X X X X X X X X X X X X X X X X

template <int K>
__device__ __forceinline__ void block(float (&r)[16], int (&ri)[16]);

#define DEF(K, OP)                                                                         \
  template <>                                                                              \
  __device__ __forceinline__ void block<K>(float (&r)[16], int (&ri)[16]) {               \
    asm volatile(OP                                                                        \
                 : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]),  \
                   "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9]), "+v"(r[10]), "+v"(r[11]), \
                   "+v"(r[12]), "+v"(r[13]), "+v"(r[14]), "+v"(r[15])                       \
                 : "v"(ri[0]));                                                            \
  }
#define L16(I)                                                                              \
  I " %0, %0, %0\n" I " %1, %1, %1\n" I " %2, %2, %2\n" I " %3, %3, %3\n" I " %4, %4, %4\n"     \
  I " %5, %5, %5\n" I " %6, %6, %6\n" I " %7, %7, %7\n" I " %8, %8, %8\n" I " %9, %9, %9\n"     \
  I " %10, %10, %10\n" I " %11, %11, %11\n" I " %12, %12, %12\n" I " %13, %13, %13\n"            \
  I " %14, %14, %14\n" I " %15, %15, %15\n"
#define U16(I)                                                                              \
  I " %0, %0\n" I " %1, %1\n" I " %2, %2\n" I " %3, %3\n" I " %4, %4\n" I " %5, %5\n"             \
  I " %6, %6\n" I " %7, %7\n" I " %8, %8\n" I " %9, %9\n" I " %10, %10\n" I " %11, %11\n"          \
  I " %12, %12\n" I " %13, %13\n" I " %14, %14\n" I " %15, %15\n"
#define T16(I)                                                                              \
  I " %0, %0, %0, %0\n" I " %1, %1, %1, %1\n" I " %2, %2, %2, %2\n" I " %3, %3, %3, %3\n"         \
  I " %4, %4, %4, %4\n" I " %5, %5, %5, %5\n" I " %6, %6, %6, %6\n" I " %7, %7, %7, %7\n"         \
  I " %8, %8, %8, %8\n" I " %9, %9, %9, %9\n" I " %10, %10, %10, %10\n" I " %11, %11, %11, %11\n"  \
  I " %12, %12, %12, %12\n" I " %13, %13, %13, %13\n" I " %14, %14, %14, %14\n"                    \
  I " %15, %15, %15, %15\n"

DEF(0, L16("v_mul_f32"))
DEF(1, T16("v_fma_f32"))
DEF(2, U16("v_cvt_f32_i32"))
DEF(3, U16("v_trunc_f32"))
DEF(4, U16("v_exp_f32"))
DEF(5, L16("v_cvt_pk_bf16_f32"))
DEF(6, T16("v_max3_f32"))
DEF(7, U16("v_exp_f16"))
DEF(8, T16("v_pk_fma_f16"))
DEF(9, L16("v_pk_add_f16"))
DEF(10, L16("v_dot2c_f32_f16"))
DEF(11, T16("v_fma_mixlo_f16"))
DEF(12, L16("v_max_f32"))
DEF(13, U16("v_mov_b32"))
DEF(14, L16("v_add_u32"))
DEF(15, U16("v_cvt_f32_f16"))

// packed-fp32 kinds: 8 independent 64-bit register pairs, each instruction used twice per block
#define DEF64(K, OP)                                                                       \
  template <>                                                                              \
  __device__ __forceinline__ void block<K>(float (&r)[16], int (&ri)[16]) {               \
    double d[8];                                                                           \
    for (int i = 0; i < 8; ++i) d[i] = __builtin_bit_cast(double, (float __attribute__((ext_vector_type(2)))){r[2 * i], r[2 * i + 1]}); \
    asm volatile(OP OP                                                                     \
                 : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]),  \
                   "+v"(d[6]), "+v"(d[7]));                                                \
    for (int i = 0; i < 8; ++i) {                                                          \
      auto v = __builtin_bit_cast(float __attribute__((ext_vector_type(2))), d[i]);        \
      r[2 * i] = v[0]; r[2 * i + 1] = v[1];                                                \
    }                                                                                      \
  }
#define L8(I)                                                                               \
  I " %0, %0, %0\n" I " %1, %1, %1\n" I " %2, %2, %2\n" I " %3, %3, %3\n" I " %4, %4, %4\n"     \
  I " %5, %5, %5\n" I " %6, %6, %6\n" I " %7, %7, %7\n"
#define T8(I)                                                                               \
  I " %0, %0, %0, %0\n" I " %1, %1, %1, %1\n" I " %2, %2, %2, %2\n" I " %3, %3, %3, %3\n"         \
  I " %4, %4, %4, %4\n" I " %5, %5, %5, %5\n" I " %6, %6, %6, %6\n" I " %7, %7, %7, %7\n"
DEF64(16, L8("v_pk_mul_f32"))
DEF64(17, L8("v_pk_add_f32"))
DEF64(18, T8("v_pk_fma_f32"))
DEF(19, U16("v_cvt_f32_bf16"))
DEF(20, T16("v_med3_f32"))
DEF(21, T16("v_dot2_f32_bf16"))

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int K>
__global__ __launch_bounds__(512) void ubench_kernel(long long* out, int iters, int mfma_waves) {
  float r[16];
  int ri[16];
  for (int i = 0; i < 16; ++i) { r[i] = 1.0f + 1e-3f * (threadIdx.x + i); ri[i] = i; }
  const int wave = threadIdx.x >> 6;
  // waves [0, mfma_waves) of the workgroup run int8 MFMAs instead (co-residence experiments);
  // the workgroup's waves are spread over the 4 SIMDs, so wave w and w+4 share a SIMD
  const bool do_mfma = (wave / 4) < mfma_waves;
  long long t0 = __builtin_amdgcn_s_memtime();
  if (do_mfma) {
    v4i a = {1, 2, 3, 4};
    v16i c = v16i{};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 16; ++j) c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c, 0, 0, 0);
    }
    r[0] += (float)c[0];
  } else {
    for (int it = 0; it < iters; ++it) block<K>(r, ri);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += r[i];
  if ((threadIdx.x & 63) == 0) {
    out[2 * (blockIdx.x * (blockDim.x >> 6) + wave)] = t1 - t0;
    out[2 * (blockIdx.x * (blockDim.x >> 6) + wave) + 1] = (long long)s;
  }
}

extern "C" int ubench(int kind, int waves_per_simd, int mfma_waves, int iters, long long* out,
                      int nblocks) {
  dim3 grid(nblocks), block(64 * 4 * waves_per_simd);
#define K(N) case N: hipLaunchKernelGGL((ubench_kernel<N>), grid, block, 0, 0, out, iters, mfma_waves); break;
  switch (kind) { K(0) K(1) K(2) K(3) K(4) K(5) K(6) K(7) K(8) K(9) K(10) K(11) K(12) K(13) K(14) K(15) K(16) K(17) K(18) K(19) K(20) K(21) }
#undef K
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
