// Co-execution microbenchmark (dev tool).  ONE workgroup per CU (forced by a 96 KiB LDS
// allocation), 4*W waves = W waves per SIMD.  Each wave loops over a block of NM int8 MFMAs
// (32x32x32, 4 accumulator chains) and NV VALU ops (16 independent v_fma_f32 chains), interleaved.
// SPLIT: waves 0..3 (one per SIMD) run only the MFMAs, the others only the VALU (role split).
// Reports cycles per iteration for every wave (s_memtime).
#include <hip/hip_runtime.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int NM, int NV, bool SPLIT>
__global__ __launch_bounds__(1024) void coexec_kernel(long long* out, int iters) {
  extern __shared__ char lds[];
  float r[16];
  for (int i = 0; i < 16; ++i) r[i] = 1.0f + 1e-3f * (threadIdx.x + i);
  v4i a = {1 + (int)threadIdx.x, 2, 3, (int)threadIdx.x};
  v16i c[4];
  for (int j = 0; j < 4; ++j) c[j] = v16i{};
  const int wave = threadIdx.x >> 6;
  const bool do_m = !SPLIT || wave < 4;
  const bool do_v = !SPLIT || wave >= 4;
  lds[threadIdx.x] = 0;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  if (do_m && do_v) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        c[m & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c[m & 3], 0, 0, 0);
#pragma unroll
        for (int v = 0; v < NV / NM; ++v) r[v & 15] = fmaf(r[v & 15], 1.0001f, 0.5f);
      }
    }
  } else if (do_m) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < NM; ++m) c[m & 3] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c[m & 3], 0, 0, 0);
    }
  } else {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int v = 0; v < NV; ++v) r[v & 15] = fmaf(r[v & 15], 1.0001f, 0.5f);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = lds[(threadIdx.x + 1) & 1023];
  for (int i = 0; i < 16; ++i) s += r[i];
  for (int j = 0; j < 4; ++j) s += (float)c[j][0];
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x >> 6) + wave;
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = (long long)s;
  }
}

extern "C" int coexec(int kind, int waves_per_simd, int iters, long long* out, int nblocks) {
  dim3 grid(nblocks), block(64 * 4 * waves_per_simd);
  const int lds = 96 * 1024;
#define K(N, NM, NV, SP)                                                                          \
  case N:                                                                                         \
    hipFuncSetAttribute((const void*)coexec_kernel<NM, NV, SP>,                                   \
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);                         \
    hipLaunchKernelGGL((coexec_kernel<NM, NV, SP>), grid, block, lds, 0, out, iters);             \
    break;
  switch (kind) {
    K(0, 12, 0, true)      // MFMA only (waves 0-3), others idle-ish (NV=0 loop)
    K(1, 12, 144, false)   // every wave: 12 MFMA + 144 VALU interleaved
    K(2, 12, 144, true)    // split: waves 0-3 MFMA, others 144 VALU
    K(3, 12, 0, false)     // every wave MFMA only
    K(4, 4, 144, false)    // hmm: NV/NM = 36 per MFMA
  }
#undef K
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
