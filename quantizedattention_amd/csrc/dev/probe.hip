// Fragment-layout probes: one-wave GEMM tiles that load operands with the lane maps assumed in
// common.h and store C with the assumed C/D map.  tests/test_gpu_layout.py checks them against a
// CPU matmul on asymmetric integer data (cdna_hip_programming.md §3: "A=I-check with ASYMMETRIC B").
#include "../common.h"
#include "qattn_dev.h"

namespace qattn {

// C[32x32] (i32, row-major) = A[32x32] (i8, row-major [m][k]) * B[32x32] (i8, row-major [k][n])
__global__ void probe_mfma_i8_kernel(const int8_t* A, const int8_t* B, int* C) {
  const int l = threadIdx.x, h = l >> 5, c = l & 31;
  v4i a, b;
  int8_t* ap = reinterpret_cast<int8_t*>(&a);
  int8_t* bp = reinterpret_cast<int8_t*>(&b);
  for (int j = 0; j < 16; ++j) {
    ap[j] = A[c * 32 + 16 * h + j];
    bp[j] = B[(16 * h + j) * 32 + c];
  }
  v16i acc = mfma_i8(a, b, v16i{});
  for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + c] = acc[r];
}

// C[32x32] (f32) = A[32x16] (f16 [m][k]) * B[16x32] (f16 [k][n])
__global__ void probe_mfma_f16_kernel(const _Float16* A, const _Float16* B, float* C) {
  const int l = threadIdx.x, h = l >> 5, c = l & 31;
  v8h a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = A[c * 16 + 8 * h + j];
    b[j] = B[(8 * h + j) * 32 + c];
  }
  v16f acc = mfma_f16(a, b, v16f{});
  for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + c] = acc[r];
}

// ds_read_b64_tr_b16 probe: M [16 rows][64 cols] u16 in LDS (row-major, 128 B rows); lane l of
// group g reads the 4x16 block rows 4*(g&3).. , cols 16*(g)...; output [64 lanes][4].
__global__ void probe_tr16_kernel(const unsigned short* M, unsigned short* out) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[16 * 64];
  const int l = threadIdx.x;
  for (int i = l; i < 16 * 64; i += 64) lds[i] = M[i];
  __syncthreads();
  const int g = l >> 4, i = l & 15;
  const int row = 4 * g + (i >> 2), col = 16 * g + 4 * (i & 3);
  v4s r = ds_read_tr16(&lds[row * 64 + col]);
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = (unsigned short)r[j];
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_probe_mfma_i8(const void* A, const void* B, void* C, void* stream) {
  hipLaunchKernelGGL(probe_mfma_i8_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const int8_t*)A, (const int8_t*)B, (int*)C);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
extern "C" int qattn_probe_mfma_f16(const void* A, const void* B, void* C, void* stream) {
  hipLaunchKernelGGL(probe_mfma_f16_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const _Float16*)A, (const _Float16*)B, (float*)C);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
extern "C" int qattn_probe_tr16(const void* M, void* out, void* stream) {
  hipLaunchKernelGGL(probe_tr16_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const unsigned short*)M, (unsigned short*)out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// packed-half helper probe: out[2i..2i+1] = {exp2_pk(x), trunc_pk(x*127)} per pair
namespace qattn {
__global__ void probe_pk_kernel(const v2h* x, v2h* e, v2h* t) {
  const int i = threadIdx.x;   // 16 lanes x 4 pairs
  if (i >= 16) return;
  const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
  v2h xi[4], xs[4], r[4];
  for (int j = 0; j < 4; ++j) { xi[j] = x[4 * i + j]; xs[j] = xi[j] * k127; }
  exp2_pk4(xi, r);
  for (int j = 0; j < 4; ++j) e[4 * i + j] = r[j];
  trunc_pk4(xs, r);
  for (int j = 0; j < 4; ++j) t[4 * i + j] = r[j];
}
}  // namespace qattn
extern "C" int qattn_probe_pk(const void* x, void* e, void* t, void* stream) {
  hipLaunchKernelGGL(probe_pk_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const v2h*)x,
                     (v2h*)e, (v2h*)t);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// int8-forward softmax helpers: w = p_operand8(e, sp) and d = fma_mix8(a, c, n), 16 lanes x 8 pairs
namespace qattn {
__global__ void probe_fwd_helpers_kernel(const v2h* e, const _Float16* sp, v2h* w, const float* a,
                                         const float* cn, v2h* d) {
  const int i = threadIdx.x;
  if (i >= 16) return;
  v2h ei[8], wo[8], dd[8];
  for (int j = 0; j < 8; ++j) ei[j] = e[8 * i + j];
  const _Float16 s = sp[i];
  const v2h sp2 = {s, s};
  const _Float16 ns = (_Float16)(-1024.0f) * s;
  const v2h nsp2 = {ns, ns};
  p_operand8(ei, sp2, nsp2, wo);
  for (int j = 0; j < 8; ++j) w[8 * i + j] = wo[j];
  float af[16];
  for (int j = 0; j < 16; ++j) af[j] = a[16 * i + j];
  fma_mix8(af, cn[2 * i], cn[2 * i + 1], dd);
  for (int j = 0; j < 8; ++j) d[8 * i + j] = dd[j];
}
}  // namespace qattn
extern "C" int qattn_probe_fwd_helpers(const void* e, const void* sp, void* w, const void* a,
                                       const void* cn, void* d, void* stream) {
  hipLaunchKernelGGL(probe_fwd_helpers_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const v2h*)e, (const _Float16*)sp, (v2h*)w, (const float*)a, (const float*)cn,
                     (v2h*)d);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// MX-FP4 probes (layout of the block-scaled MFMA operands and of the fp4 converts):
//   mfma_fp4: one wave, A / B as 64 lanes x 16 bytes (32 e2m1 nibbles, low nibble first), one
//   e8m0 scale byte per lane (byte 0 of sa / sb), C = 64 lanes x 16 f32.
//   fp4_cvt: lane i packs x[8i .. 8i+7] with v_cvt_scalef32_pk_fp4_f32 (scale s[i]) into one dword
//   and decodes it back with v_cvt_scalef32_pk_f32_fp4 (same scale).
namespace qattn {
typedef int v8i_ __attribute__((ext_vector_type(8)));
__global__ void probe_mfma_fp4_kernel(const v4i* A, const v4i* B, const unsigned* sa, const unsigned* sb,
                                      v16f* C) {
  const int l = threadIdx.x;
  const v4i a4 = A[l], b4 = B[l];
  const v8i_ a = {a4[0], a4[1], a4[2], a4[3], 0, 0, 0, 0};
  const v8i_ b = {b4[0], b4[1], b4[2], b4[3], 0, 0, 0, 0};
  C[l] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, v16f{}, 4, 4, 0, (int)sa[l], 0, (int)sb[l]);
}
__global__ void probe_fp4_cvt_kernel(const float* x, const float* s, unsigned* packed, float* back) {
  const int i = threadIdx.x;
  unsigned w = 0;
  w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, x[8 * i + 0], x[8 * i + 1], s[i], 0);
  w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, x[8 * i + 2], x[8 * i + 3], s[i], 1);
  w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, x[8 * i + 4], x[8 * i + 5], s[i], 2);
  w = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(w, x[8 * i + 6], x[8 * i + 7], s[i], 3);
  packed[i] = w;
#define QA_BACK(j)                                                          \
  {                                                                         \
    const auto r = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(w, s[i], j);    \
    back[8 * i + 2 * j] = r[0];                                             \
    back[8 * i + 2 * j + 1] = r[1];                                         \
  }
  QA_BACK(0) QA_BACK(1) QA_BACK(2) QA_BACK(3)
#undef QA_BACK
}
}  // namespace qattn
extern "C" int qattn_probe_mfma_fp4(const void* A, const void* B, const void* sa, const void* sb, void* C,
                                    void* stream) {
  hipLaunchKernelGGL(probe_mfma_fp4_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const v4i*)A,
                     (const v4i*)B, (const unsigned*)sa, (const unsigned*)sb, (v16f*)C);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
extern "C" int qattn_probe_fp4_cvt(const void* x, const void* s, void* packed, void* back, void* stream) {
  hipLaunchKernelGGL(probe_fp4_cvt_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)x,
                     (const float*)s, (unsigned*)packed, (float*)back);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// The int8 quantiser's division-free index (common.h quant8) against the IEEE fp32 division of the
// reference, trunc(RNE_f16(fp32(x) / s)), for every finite fp16 x with |x| < 127.5 s (the range a
// block with scale s = f16(amax / 127) can hold; other x are replaced by 0) and every fp16 scale
// s in [s_lo, s_hi) (bit patterns).  Thread: 8 consecutive x bit patterns; grid.y strides over s.
// Mismatching bytes or image values are counted in bad[0] (vector atomics, only on a mismatch);
// bad[1..5] hold the first one found.
namespace qattn {
__global__ __launch_bounds__(256) void probe_quant_div_kernel(int s_lo, int s_hi, unsigned* bad) {
  const unsigned x0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  for (int sb = s_lo + (int)blockIdx.y; sb < s_hi; sb += (int)gridDim.y) {
    const float s = (float)__builtin_bit_cast(_Float16, (unsigned short)sb);
    v8h x;
    int ref[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      _Float16 xv = __builtin_bit_cast(_Float16, (unsigned short)(x0 + j));
      const float xf = (float)xv;
      if (!(fabsf(xf) < 127.5f * s)) xv = (_Float16)0.0f;   // (also NaN / inf)
      x[j] = xv;
      ref[j] = s != 0.f ? (int)__builtin_truncf((float)(_Float16)((float)xv / s)) : 0;
    }
    unsigned lo, hi;
    float qf[8];
    quant8(x, s, quant_rcp(s), lo, hi, qf);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int byte = (int)(signed char)(((j < 4 ? lo : hi) >> (8 * (j & 3))) & 0xff);
      if ((byte != ref[j]) || (__float_as_uint(qf[j]) != __float_as_uint((float)ref[j]))) {
        // bad[0]: count; bad[1..5]: the first mismatch (s bits, x bits, reference, byte, image bits)
        if (atomicAdd(bad, 1u) == 0) {
          bad[1] = (unsigned)sb;
          const _Float16 xj = x[j];   // (not bit_cast of the element lvalue: hipcc folds it to x[0])
          bad[2] = (unsigned)__builtin_bit_cast(unsigned short, xj);
          bad[3] = (unsigned)ref[j];
          bad[4] = (unsigned)byte;
          bad[5] = __float_as_uint(qf[j]);
        }
      }
    }
  }
}
}  // namespace qattn
extern "C" int qattn_probe_quant_div(int s_lo, int s_hi, void* bad, void* stream) {
  hipLaunchKernelGGL(probe_quant_div_kernel, dim3(65536 / 8 / 256, 1024), dim3(256), 0, (hipStream_t)stream,
                     s_lo, s_hi, (unsigned*)bad);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// A device copy by a FIXED number of workgroups (grid-stride, 16 B per lane and step): a stand-in for
// an RCCL collective kernel, which moves its bytes with a few persistent workgroups (one per
// channel), next to a grid-filling copy (tools/overlap_probe.py).
__global__ __launch_bounds__(256) void few_wg_copy_kernel(const uint4* __restrict__ src,
                                                          uint4* __restrict__ dst, long n16) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}
extern "C" int qattn_probe_few_wg_copy(const void* src, void* dst, long bytes, int workgroups,
                                       void* stream) {
  if (bytes % 16 != 0 || workgroups < 1) return 1;
  hipLaunchKernelGGL(few_wg_copy_kernel, dim3((unsigned)workgroups), dim3(256), 0, (hipStream_t)stream,
                     (const uint4*)src, (uint4*)dst, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// exp2 on the fp16 domain: for every fp16 bit pattern h, e32[h] = v_exp_f32((float)h) and
// e16[h] = v_exp_f16(h) (bits).  tools/exp2_probe.py compares them with the correctly rounded
// values (the literal P chain of the int8 forward evaluates exp2 only at fp16 arguments).
namespace qattn {
__global__ __launch_bounds__(256) void probe_exp2_dom_kernel(unsigned* e32, unsigned short* e16) {
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  const _Float16 h = __builtin_bit_cast(_Float16, (unsigned short)i);
  e32[i] = __float_as_uint(exp2_f32((float)h));
  v2h x[4] = {{h, h}, {h, h}, {h, h}, {h, h}}, r[4];
  exp2_pk4(x, r);
  e16[i] = __builtin_bit_cast(unsigned short, r[0][1]);
}
}  // namespace qattn
extern "C" int qattn_probe_exp2_dom(void* e32, void* e16, void* stream) {
  hipLaunchKernelGGL(probe_exp2_dom_kernel, dim3(65536 / 256), dim3(256), 0, (hipStream_t)stream,
                     (unsigned*)e32, (unsigned short*)e16);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
