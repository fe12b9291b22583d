// Overlap microbenchmark (dev tool): W waves per SIMD each loop over a block of NM int8 MFMAs
// (32x32x32, NA independent accumulator chains) and NV independent VALU ops (v_mul_f32 on 16
// registers, or v_exp_f16 when EXP).  Reports cycles per iteration per wave: compare with the
// MFMA-only (NV=0) and VALU-only (NM=0) runs to see how far the two pipes overlap.
#include <hip/hip_runtime.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int NM, int NA, int NV, bool INTERLEAVE>
__global__ __launch_bounds__(1024) void overlap_kernel(long long* out, int iters) {
  float r[16];
  for (int i = 0; i < 16; ++i) r[i] = 1.0f + 1e-3f * (threadIdx.x + i);
  v4i a = {1, 2, 3, (int)threadIdx.x};
  v16i c[NA];
  for (int j = 0; j < NA; ++j) c[j] = v16i{};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (INTERLEAVE) {
      // NV/NM VALU ops after each MFMA
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        c[m % NA] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c[m % NA], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < NV / (NM ? NM : 1); ++v) r[v & 15] = r[v & 15] * 1.0001f;
      }
    } else {
#pragma unroll
      for (int m = 0; m < NM; ++m) c[m % NA] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c[m % NA], 0, 0, 0);
#pragma unroll
      for (int v = 0; v < NV; ++v) r[v & 15] = r[v & 15] * 1.0001f;
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += r[i];
  for (int j = 0; j < NA; ++j) s += (float)c[j][0];
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = (long long)s;
  }
}

extern "C" int overlap(int kind, int waves_per_simd, int iters, long long* out, int nblocks) {
  dim3 grid(nblocks), block(64 * 4 * waves_per_simd);
#define K(N, NM, NA, NV, IL) case N: hipLaunchKernelGGL((overlap_kernel<NM, NA, NV, IL>), grid, block, 0, 0, out, iters); break;
  switch (kind) {
    K(0, 12, 4, 0, false)
    K(1, 0, 1, 128, false)
    K(2, 12, 4, 128, false)
    K(3, 12, 4, 128, true)
    K(4, 12, 1, 0, false)
    K(5, 12, 1, 128, true)
    K(6, 12, 4, 64, true)
    K(7, 0, 1, 64, false)
  }
#undef K
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
