// bf16 FlashAttention forward with the "multiple-max" beta correction (arXiv 2510.04212) for
// gfx950; replaces helion_atten_bf16_fwd_training (attention_bf16.py:107-296).
//
// Numerics: the reference's eager rounding contract at the reference's
// pinned k-tile KT = 16 (bf16:736), applied sequentially per 16-key sub-tile:
//   S  = bf16(fp16(q.k))                (fp16 MFMA, fp32 accumulate)          bf16:215-216
//   causal: S = (q - k > 0) ? S : -126                                          bf16:222-233
//   m' = bf16(max(m, bf16(rowmax S * qks)))                                     bf16:236-239
//   if #{S >= bf16(m' - bf16(1e-3))} > 1: m' = 2m' (m'>0) | 0 (m'<0)            bf16:248-264
//   P  = bf16(exp2(bf16(bf16(S*qks) - m')));  r = bf16(exp2(bf16(m - m')))       bf16:267-276
//   l  = l*r + sum P;  O = O*r + P.V  (bf16 MFMA, fp32 accumulate)              bf16:279-285
//   lse = m + log2 l;  O /= l                                                   bf16:288-294
//
// Structure (same as int8_attn_fwd.hip): 4 waves x 32 query rows per workgroup, keys streamed in
// 64-key blocks through a 2-stage LDS ring, swapped QK^T (keys in registers, one query per lane
// pair), P fed straight from the accumulator registers into the PV MFMA (B operand), V read
// column-wise with ds_read_b64_tr_b16.  One 16-key sub-tile == one k-step of the 32x32x16 PV MFMA.
#include "common.h"

namespace qattn {

template <int D>
struct Bf16FwdCfg {
  static constexpr int KB = 64;
  static constexpr int ROWB = 2 * D;            // bytes per K/V row
  static constexpr int NCH = ROWB / 16;         // 16-B chunks per row
  static constexpr int TILE = KB * ROWB;        // bytes per K (or V) block
  static constexpr int STAGE = 2 * TILE;
  static constexpr int NKS = D / 16;            // f16 k-steps for QK^T
  static constexpr int NDB = D / 32;
  static constexpr int LOADS = TILE / (256 * 16);
  static constexpr int K_SHIFT = (D == 128) ? 0 : 1;   // swizzle = (row >> K_SHIFT) & (NCH-1)
  static constexpr int V_SHIFT = (D == 128) ? 2 : 1;   // swizzle = (row & 3) << V_SHIFT
};

template <int D>
QA_DEVICE int kf_off(int row, int ch) {
  using C = Bf16FwdCfg<D>;
  return row * C::ROWB + 16 * (ch ^ ((row >> C::K_SHIFT) & (C::NCH - 1)));
}
template <int D>
QA_DEVICE int vf_off(int row, int ch) {
  using C = Bf16FwdCfg<D>;
  return row * C::ROWB + 16 * (ch ^ ((row & 3) << C::V_SHIFT));
}

// A operand (V^T, 32 d x 16 keys) of one PV k-step via two transposed reads.
template <int D, typename T8>
QA_DEVICE T8 load_vt_frag(const char* vl, int key_base, int b, int lane) {
  const int h = lane >> 5, gg = (lane >> 4) & 1, i16 = lane & 15;
  const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
  const int key = key_base + 4 * h + (i16 >> 2);
  const int ch = d / 8, within = (d % 8) * 2;
  const v8s a = ds_read_tr16_x2(vl + vf_off<D>(key, ch) + within,
                                vl + vf_off<D>(key + 8, ch) + within);
  return __builtin_bit_cast(T8, a);
}

template <int D>
__global__ __launch_bounds__(256, 2) void bf16_fwd_kernel(
    const _Float16* __restrict__ q, const _Float16* __restrict__ k, const __bf16* __restrict__ v,
    float* __restrict__ out, float* __restrict__ lse, int BH, int Sq, int Sk, int causal, float qks) {
  using C = Bf16FwdCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nq = (Sq + 127) / 128;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qt * 128 + wave * 32;
  const bool active = q0 < Sq;
  const int qidx = q0 + c32;                     // this lane's query row
  const float thr_eps = 0.00099945068359375f;  // bf16(1e-3): eager `bf16 - 1e-3` rounds the scalar (bf16:248)

  v8h qf[C::NKS];
  if (active) {
    const _Float16* qrow = q + ((long)bh * Sq + qidx) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v8h*>(qrow + 16 * s);
  }
  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  float m = -INFINITY;   // bf16-valued
  float l = 1.0f;

  const char* kbase = reinterpret_cast<const char*>(k + (long)bh * Sk * D);
  const char* vbase = reinterpret_cast<const char*>(v + (long)bh * Sk * D);
  const int nkb = (Sk + C::KB - 1) / C::KB;

  v4i kst[C::LOADS], vst[C::LOADS];
  auto stage_load = [&](int kb) {
    const int key0 = kb * C::KB;
#pragma unroll
    for (int i = 0; i < C::LOADS; ++i) {
      const int e = i * 256 + tid, row = e / C::NCH, ch = e % C::NCH;
      const bool ok = key0 + row < Sk;
      const long off = (long)(key0 + row) * C::ROWB + 16 * ch;
      kst[i] = ok ? *reinterpret_cast<const v4i*>(kbase + off) : v4i{0, 0, 0, 0};
      vst[i] = ok ? *reinterpret_cast<const v4i*>(vbase + off) : v4i{0, 0, 0, 0};
    }
  };
  auto stage_store = [&](int buf) {
    char* kl = smem + buf * C::STAGE;
    char* vl = kl + C::TILE;
#pragma unroll
    for (int i = 0; i < C::LOADS; ++i) {
      const int e = i * 256 + tid, row = e / C::NCH, ch = e % C::NCH;
      *reinterpret_cast<v4i*>(kl + kf_off<D>(row, ch)) = kst[i];
      *reinterpret_cast<v4i*>(vl + vf_off<D>(row, ch)) = vst[i];
    }
  };

  stage_load(0);
  stage_store(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) stage_load(kb + 1);
    const char* kl = smem + (kb & 1) * C::STAGE;
    const char* vl = kl + C::TILE;
    const int ntile = min(2, (Sk - kb * C::KB) / 32);
    if (active) {
      for (int u = 0; u < ntile; ++u) {
        const int key_t0 = kb * C::KB + 32 * u;
        v16f acc = v16f{};
#pragma unroll
        for (int s = 0; s < C::NKS; ++s) {
          const v8h kf = *reinterpret_cast<const v8h*>(kl + kf_off<D>(32 * u + c32, 2 * s + h));
          acc = mfma_f16(kf, qf[s], acc);
        }
        // S = bf16(fp16(acc)); causal fill -126 where q - k <= 0
        const bool need_mask = causal && (key_t0 + 31 >= q0);  // some (q, key) of the tile has q - key <= 0
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float s = rne_bf16((float)(_Float16)acc[i]);
          if (need_mask) {
            const int key = key_t0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (qidx - key <= 0) s = -126.0f;
          }
          acc[i] = s;
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          float rl = -INFINITY;
#pragma unroll
          for (int j = 0; j < 8; ++j) rl = fmaxf(rl, acc[8 * t + j]);
          const float rmax = fmaxf(rl, xor32_f(rl));
          float nm = fmaxf(m, rne_bf16(rmax * qks));
          const float thr = rne_bf16(nm - thr_eps);
          int cl = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) cl += (acc[8 * t + j] >= thr) ? 1 : 0;
          const int cnt = cl + __shfl_xor(cl, 32);
          if (cnt > 1) {
            if (nm > 0.f) nm = rne_bf16(2.0f * nm);
            else if (nm < 0.f) nm = 0.f;
          }
          float lt = 0.f;
          float p[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            p[j] = rne_bf16(exp2_f32(rne_bf16(rne_bf16(acc[8 * t + j] * qks) - nm)));
            lt += p[j];
          }
          lt += xor32_f(lt);
          const float r = rne_bf16(exp2_f32(rne_bf16(m - nm)));
          m = nm;
          l = l * r + lt;
          if (__ballot(r != 1.0f)) {
#pragma unroll
            for (int b = 0; b < C::NDB; ++b) o[b] *= r;
          }
          v4u pk;
#pragma unroll
          for (int j = 0; j < 4; ++j) pk[j] = pk_bf16(p[2 * j], p[2 * j + 1]);
          const v8bf pb = __builtin_bit_cast(v8bf, pk);
#pragma unroll
          for (int b = 0; b < C::NDB; ++b) {
            const v8bf a = load_vt_frag<D, v8bf>(vl, 32 * u + 16 * t, b, lane);
            o[b] = mfma_bf16(a, pb, o[b]);
          }
        }
      }
    }
    if (kb + 1 < nkb) stage_store((kb + 1) & 1);
    __syncthreads();
  }
  if (!active) return;
  const long row = (long)bh * Sq + qidx;
  if (h == 0) lse[row] = m + log2_f32(l);
  float* orow = out + row * D;
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4f w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = o[b][4 * g + j] / l;
      *reinterpret_cast<v4f*>(orow + 32 * b + 8 * g + 4 * h) = w;
    }
  }
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_bf16_fwd(const void* q, const void* k, const void* v, void* out, void* lse, long bh,
                              long sq, long sk, int head_dim, int causal, float qks, void* stream) {
  if (sq % 32 != 0 || sk % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0 || sq == 0) return 0;
  const int nq = (int)((sq + 127) / 128);
  dim3 grid((unsigned)(nq * bh)), block(256);
  hipStream_t st = (hipStream_t)stream;
#define QA_LAUNCH(Dv)                                                                          \
  hipLaunchKernelGGL((bf16_fwd_kernel<Dv>), grid, block, 2 * Bf16FwdCfg<Dv>::STAGE, st,        \
                     (const _Float16*)q, (const _Float16*)k, (const __bf16*)v, (float*)out,      \
                     (float*)lse, (int)bh, (int)sq, (int)sk, causal, qks)
  if (head_dim == 128) QA_LAUNCH(128); else QA_LAUNCH(64);
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
