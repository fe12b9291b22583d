// Forward-mode tangent attention for gfx950; replaces helion_attention_jvp_forward_fp32
// (attention_jvp.py:24-195).  With P = softmax(q k^T * sm) and tS = (tq k^T + q tk^T) * sm:
//   H = P o tS,   tO = (P tV + H V - rowsum(H) * O) / l     (jvp:148-190, Appendix A.3)
// computed online over key tiles with the usual running-max rescale applied to every accumulator.
// A = P tV and B = H V only ever appear as A + B, so one accumulator (AB) holds both:
//   AB^T[d][q] += tV^T P^T + V^T H^T    (two MFMA chains into the same registers).
// Per 32-key tile and wave: S^T (8), tS^T (16), O^T (8), AB^T (16) v_mfma_f32_32x32x16_bf16 at
// D = 128 -> the 12*S^2*D FLOP of SURVEY §8d.  bf16 operands (inputs bf16 exact; P and H rounded to
// bf16 for the PV-type products), fp32 accumulation and fp32 softmax state.
//
// K, tK (row-read images) and V, tV (transposed-read images) are staged by LDS-DMA
// (global_load_lds_dwordx4, swizzle applied on the per-lane source address, LDS destination
// lane-linear), 64 keys per stage, 2 stages (128 KiB): no staging registers, which the 4 fp32
// accumulators of this kernel cannot spare.
#include "common.h"

namespace qattn {

template <int D>
struct JvpCfg {
  static constexpr int KB = 64;
  static constexpr int ROWB = 2 * D;
  static constexpr int NCH = ROWB / 16;
  static constexpr int TILE = KB * ROWB;
  static constexpr int STAGE = 4 * TILE;  // K, tK, V, tV
  static constexpr int NKS = D / 16;
  static constexpr int NDB = D / 32;
};
template <int D>
QA_DEVICE int jrow_sw(int row) { return (D == 128) ? (row & 15) : ((row >> 1) & 7); }
template <int D>
QA_DEVICE int jtr_sw(int row) { return (row & 3) << ((D == 128) ? 2 : 1); }

// LDS-DMA one [64 rows][ROWB] tile: lane-linear destination, swizzled source chunk.
template <int D, bool TR>
QA_DEVICE void dma_tile(const char* gsrc, char* lds_tile, int wave, int lane) {
  using C = JvpCfg<D>;
  constexpr int RPI = 64 / C::NCH;       // rows per wave-instruction (1 KiB)
  constexpr int IPW = C::NCH / 4;        // instructions per wave (4 waves)
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int inst = wave * IPW + i;
    const int row = inst * RPI + lane / C::NCH;
    const int p = lane % C::NCH;
    const int ch = p ^ (TR ? jtr_sw<D>(row) : jrow_sw<D>(row));
    glds16(gsrc + (long)row * C::ROWB + 16 * ch, lds_tile + inst * 1024);
  }
}

template <int D>
QA_DEVICE v8bf jtr_frag(const char* base, int row_base, int b, int lane) {
  using C = JvpCfg<D>;
  const int h = lane >> 5, gg = (lane >> 4) & 1, i16 = lane & 15;
  const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
  const int row = row_base + 4 * h + (i16 >> 2);
  const int ch = d / 8, within = (d % 8) * 2;
  return __builtin_bit_cast(
      v8bf, ds_read_tr16_x2(base + row * C::ROWB + 16 * (ch ^ jtr_sw<D>(row)) + within,
                            base + (row + 8) * C::ROWB + 16 * (ch ^ jtr_sw<D>(row + 8)) + within));
}

template <int D>
__global__ __launch_bounds__(256, 1) void jvp_fwd_kernel(
    const __bf16* __restrict__ q, const __bf16* __restrict__ k, const __bf16* __restrict__ v,
    const __bf16* __restrict__ tq, const __bf16* __restrict__ tk, const __bf16* __restrict__ tv,
    float* __restrict__ out, float* __restrict__ tout, float* __restrict__ lse, int BH, int Sq, int Sk,
    float qks, float sm) {
  using C = JvpCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nq = (Sq + 127) / 128;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qt * 128 + wave * 32;
  const bool active = q0 < Sq;
  const int qi = q0 + c32;
  v8bf qf[C::NKS], tqf[C::NKS];
  if (active) {
    const long r = (long)bh * Sq + qi;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
      qf[s] = *reinterpret_cast<const v8bf*>(q + r * D + 16 * s + 8 * h);
      tqf[s] = *reinterpret_cast<const v8bf*>(tq + r * D + 16 * s + 8 * h);
    }
  }
  v16f o[C::NDB], ab[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) { o[b] = v16f{}; ab[b] = v16f{}; }
  float m = -INFINITY, l = 0.f, racc = 0.f;   // jvp:130-134

  const long kv0 = (long)bh * Sk * D;
  const char* gk = reinterpret_cast<const char*>(k + kv0);
  const char* gtk = reinterpret_cast<const char*>(tk + kv0);
  const char* gv = reinterpret_cast<const char*>(v + kv0);
  const char* gtv = reinterpret_cast<const char*>(tv + kv0);
  const int nkb = Sk / C::KB;
  auto stage = [&](int kb, int buf) {
    char* base = smem + buf * C::STAGE;
    const long off = (long)kb * C::TILE;
    dma_tile<D, false>(gk + off, base, wave, lane);
    dma_tile<D, false>(gtk + off, base + C::TILE, wave, lane);
    dma_tile<D, true>(gv + off, base + 2 * C::TILE, wave, lane);
    dma_tile<D, true>(gtv + off, base + 3 * C::TILE, wave, lane);
  };
  stage(0, 0);
  vmem_drain();
  dma_wait_barrier();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) stage(kb + 1, (kb + 1) & 1);
    const char* base = smem + (kb & 1) * C::STAGE;
    const char* kl = base;
    const char* tkl = base + C::TILE;
    const char* vl = base + 2 * C::TILE;
    const char* tvl = base + 3 * C::TILE;
    if (active) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        v16f sacc = v16f{}, tacc = v16f{};
#pragma unroll
        for (int s = 0; s < C::NKS; ++s) {
          const int row = 32 * u + c32, ch = 2 * s + h;
          const v8bf ka = *reinterpret_cast<const v8bf*>(kl + row * C::ROWB + 16 * (ch ^ jrow_sw<D>(row)));
          const v8bf tka = *reinterpret_cast<const v8bf*>(tkl + row * C::ROWB + 16 * (ch ^ jrow_sw<D>(row)));
          sacc = mfma_bf16(ka, qf[s], sacc);
          tacc = mfma_bf16(ka, tqf[s], tacc);
          tacc = mfma_bf16(tka, qf[s], tacc);
        }
        float rl = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; ++i) rl = fmaxf(rl, sacc[i]);
        const float rmax = fmaxf(rl, xor32_f(rl));
        const float nm = fmaxf(m, rmax * qks);   // jvp:155-158
        float p[16], hh[16], lt = 0.f, rt = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          p[i] = exp2_f32(sacc[i] * qks - nm);     // jvp:160-161
          hh[i] = p[i] * (tacc[i] * sm);           // jvp:152-153,176
          lt += p[i];
          rt += hh[i];
        }
        lt += xor32_f(lt);
        rt += xor32_f(rt);
        const float rs = exp2_f32(m - nm);         // jvp:164
        l = l * rs + lt;
        racc = racc * rs + rt;                     // jvp:178
        m = nm;
        if (__ballot(rs != 1.0f)) {
#pragma unroll
          for (int b = 0; b < C::NDB; ++b) { o[b] *= rs; ab[b] *= rs; }
        }
        v8bf pb[2], hb[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v4u pp, hp;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pp[j] = pk_bf16(p[8 * s + 2 * j], p[8 * s + 2 * j + 1]);
            hp[j] = pk_bf16(hh[8 * s + 2 * j], hh[8 * s + 2 * j + 1]);
          }
          pb[s] = __builtin_bit_cast(v8bf, pp);
          hb[s] = __builtin_bit_cast(v8bf, hp);
        }
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const v8bf va = jtr_frag<D>(vl, 32 * u + 16 * s, b, lane);
            const v8bf tva = jtr_frag<D>(tvl, 32 * u + 16 * s, b, lane);
            o[b] = mfma_bf16(va, pb[s], o[b]);      // jvp:171
            ab[b] = mfma_bf16(tva, pb[s], ab[b]);   // jvp:173-174
            ab[b] = mfma_bf16(va, hb[s], ab[b]);    // jvp:180-181
          }
        }
      }
    }
    dma_wait_barrier();
  }
  if (!active) return;
  const long r = (long)bh * Sq + qi;
  if (h == 0) lse[r] = m + log2_f32(l);          // jvp:183
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4f wo, wt;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float of = o[b][4 * g + j] / l;                   // jvp:188
        wo[j] = of;
        wt[j] = (ab[b][4 * g + j] - racc * of) / l;             // jvp:190
      }
      *reinterpret_cast<v4f*>(out + r * D + 32 * b + 8 * g + 4 * h) = wo;
      *reinterpret_cast<v4f*>(tout + r * D + 32 * b + 8 * g + 4 * h) = wt;
    }
  }
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_jvp_fwd(const void* q, const void* k, const void* v, const void* tq, const void* tk,
                             const void* tv, void* out, void* tout, void* lse, long bh, long sq, long sk,
                             int head_dim, int flags, float qks, float sm, void* stream) {
  if (flags != 0 || sq % 32 != 0 || sk % 64 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0 || sq == 0) return 0;
  const int nq = (int)((sq + 127) / 128);
  hipStream_t st = (hipStream_t)stream;
#define QA_LAUNCH(Dv)                                                                              \
  {                                                                                                \
    constexpr int lds = 2 * JvpCfg<Dv>::STAGE;                                                     \
    hipFuncSetAttribute((const void*)jvp_fwd_kernel<Dv>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                        lds);                                                                      \
    hipLaunchKernelGGL((jvp_fwd_kernel<Dv>), dim3((unsigned)(nq * bh)), dim3(256), lds, st,        \
                       (const __bf16*)q, (const __bf16*)k, (const __bf16*)v, (const __bf16*)tq,    \
                       (const __bf16*)tk, (const __bf16*)tv, (float*)out, (float*)tout,            \
                       (float*)lse, (int)bh, (int)sq, (int)sk, qks, sm);                           \
  }
  if (head_dim == 128) QA_LAUNCH(128) else QA_LAUNCH(64)
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
