// Forward-mode tangent attention for gfx950; replaces helion_attention_jvp_forward_fp32
// (attention_jvp.py:24-195).  With P = softmax(q k^T * sm) and tS = (tq k^T + q tk^T) * sm:
//   H = P o tS,   tO = (P tV + H V - rowsum(H) * O) / l     (jvp:148-190, Appendix A.3)
// computed online over key tiles with the running-max rescale applied to every accumulator (deferred
// until the max grows by more than JVP_THR).
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

// X3 = the fp32-accurate mode: every fp32 operand x is carried as two bf16 images x = hi + lo
// (hi = bf16(x), lo = bf16(x - hi), qattn_split_bf16) and each product as
// hi*hi + hi*lo + lo*hi + lo*lo, exact up to the split residual |x - hi - lo| <= 2^-17 |x|.
// 4x the MFMAs of the bf16 mode.  Measured vs torch.func.jvp in float64 (tools/jvp_err.py): O within
// 6e-6, tO within 8e-6 at max|tO| = 1.35 (dropping lo*lo: tO 2.7e-5).
// TAN = false is the primal-only kernel (O and lse, no tangent chains or tangent operands): the
// forward of AttentionJVP_autograd_function.  Its S, P, l and O arithmetic is the
// same instruction sequence as the tangent kernel's, so O / lse are bit-identical to the ones
// qattn_jvp_fwd returns (tests/test_gpu_jvp.py).
// running-max deferral threshold (log2 units) of the online softmax
constexpr float JVP_THR = 8.0f;
// QA_JVP_HLO = 1 (build option, off by default): in the bf16 mode H = P tS also enters the B = H V
// product as a bf16 lo residual (hi + lo: 16 bits).  The bf16 rounding of H dominates tO's error
// at large logits: on the climbing-max input of tests/test_gpu_edge.py 0.33 -> 0.053 (max|tO| =
// 51), for 8 more MFMAs per 32 keys: config 5 0.267 -> 0.30 ms.  The fp32 (X3) mode is the
// accurate path.
#ifndef QA_JVP_HLO
#define QA_JVP_HLO 0
#endif

template <int D, bool X3, bool TAN = true>
struct JvpCfg {
  static constexpr int KB = X3 ? 32 : 64;     // keys per stage
  static constexpr int NIMG = X3 ? 2 : 1;     // bf16 images per operand
  static constexpr int ROWB = 2 * D;
  static constexpr int NCH = ROWB / 16;
  static constexpr int TILE = KB * ROWB;
  static constexpr int NOPS = TAN ? 4 : 2;    // K, tK, V, tV / K, V
  static constexpr int STAGE = NOPS * NIMG * TILE;
  static constexpr int SK = 0, STK = 1, SV = TAN ? 2 : 1, STV = 3;   // operand slots in a stage
  static constexpr int NKS = D / 16;
  static constexpr int NDB = D / 32;
};
template <int D>
QA_DEVICE int jrow_sw(int row) { return (D == 128) ? (row & 15) : ((row >> 1) & 7); }
template <int D>
QA_DEVICE int jtr_sw(int row) { return (row & 3) << ((D == 128) ? 2 : 1); }

// LDS-DMA one [KB rows][ROWB] tile: lane-linear destination, swizzled source chunk.
template <int D, bool X3, bool TR>
QA_DEVICE void dma_tile(const char* gsrc, char* lds_tile, int wave, int lane) {
  using C = JvpCfg<D, X3>;
  constexpr int RPI = 64 / C::NCH;                 // rows per wave-instruction (1 KiB)
  constexpr int IPW = C::TILE / 1024 / 4;          // instructions per wave (4 waves)
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
  constexpr int ROWB = 2 * D;
  const int h = lane >> 5, gg = (lane >> 4) & 1, i16 = lane & 15;
  const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
  const int row = row_base + 4 * h + (i16 >> 2);
  const int ch = d / 8, within = (d % 8) * 2;
  return __builtin_bit_cast(
      v8bf, ds_read_tr16_x2(base + row * ROWB + 16 * (ch ^ jtr_sw<D>(row)) + within,
                            base + (row + 8) * ROWB + 16 * (ch ^ jtr_sw<D>(row + 8)) + within));
}

// Operand images: [0] = hi (the bf16 operand itself in the bf16 mode), [1] = lo (X3 only).
struct JvpArgs {
  const __bf16* q[2];
  const __bf16* k[2];
  const __bf16* v[2];
  const __bf16* tq[2];
  const __bf16* tk[2];
  const __bf16* tv[2];
  float* out;
  float* tout;
  float* lse;
  int BH, Sq, Sk, G;   // G: query heads per key/value head (grouped-query attention)
  float qks, sm;
};

template <int D, bool X3, bool TAN>
__global__ __launch_bounds__(256, 1) void jvp_fwd_kernel(JvpArgs a) {
  using C = JvpCfg<D, X3, TAN>;
  constexpr int NI = C::NIMG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Sq = a.Sq, Sk = a.Sk;
  const float qks = a.qks, sm = a.sm;
  const int nq = (Sq + 127) / 128;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, a.BH, bh, qt);
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: `active` is a scalar branch
  const int q0 = qt * 128 + wave * 32;
  const bool active = q0 < Sq;
  const int qi = q0 + c32;
  v8bf qf[NI][C::NKS], tqf[NI][C::NKS];
  if (active) {
    const long r = (long)bh * Sq + qi;
#pragma unroll
    for (int x = 0; x < NI; ++x)
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        qf[x][s] = *reinterpret_cast<const v8bf*>(a.q[x] + r * D + 16 * s + 8 * h);
        if constexpr (TAN) tqf[x][s] = *reinterpret_cast<const v8bf*>(a.tq[x] + r * D + 16 * s + 8 * h);
      }
  }
  v16f o[C::NDB], ab[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) { o[b] = v16f{}; ab[b] = v16f{}; }
  float m = -INFINITY, l = 0.f, racc = 0.f;   // jvp:130-134

  const long kv0 = (long)(bh / a.G) * Sk * D;
  const int nkb = Sk / C::KB;
  // stage layout: [K x NI][tK x NI][V x NI][tV x NI]  (primal-only: [K x NI][V x NI])
  auto stage = [&](int kb, int buf) {
    char* base = smem + buf * C::STAGE;
    const long off = (long)kb * C::TILE;
#pragma unroll
    for (int x = 0; x < NI; ++x) {
      dma_tile<D, X3, false>(reinterpret_cast<const char*>(a.k[x] + kv0) + off, base + (C::SK * NI + x) * C::TILE, wave, lane);
      dma_tile<D, X3, true>(reinterpret_cast<const char*>(a.v[x] + kv0) + off, base + (C::SV * NI + x) * C::TILE, wave, lane);
      if constexpr (TAN) {
        dma_tile<D, X3, false>(reinterpret_cast<const char*>(a.tk[x] + kv0) + off, base + (C::STK * NI + x) * C::TILE, wave, lane);
        dma_tile<D, X3, true>(reinterpret_cast<const char*>(a.tv[x] + kv0) + off, base + (C::STV * NI + x) * C::TILE, wave, lane);
      }
    }
  };
  // hi*hi (+ hi*lo + lo*hi + lo*lo in X3): acc += A.B for split operands
  auto mm = [&](const v8bf* A, const v8bf* B, v16f acc) -> v16f {
    acc = mfma_bf16(A[0], B[0], acc);
    if constexpr (X3) {
      acc = mfma_bf16(A[0], B[1], acc);
      acc = mfma_bf16(A[1], B[0], acc);
      acc = mfma_bf16(A[1], B[1], acc);
    }
    return acc;
  };
  stage(0, 0);
  vmem_drain();
  dma_wait_barrier();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) stage(kb + 1, (kb + 1) & 1);
    const char* base = smem + (kb & 1) * C::STAGE;
    if (active) {
#pragma unroll
      for (int u = 0; u < C::KB / 32; ++u) {
        v16f sacc = v16f{}, tacc = v16f{};
#pragma unroll
        for (int s = 0; s < C::NKS; ++s) {
          const int row = 32 * u + c32, ch = 2 * s + h;
          const int off = row * C::ROWB + 16 * (ch ^ jrow_sw<D>(row));
          v8bf ka[NI], tka[NI], qq[NI], tqq[NI];
#pragma unroll
          for (int x = 0; x < NI; ++x) {
            ka[x] = *reinterpret_cast<const v8bf*>(base + (C::SK * NI + x) * C::TILE + off);
            if constexpr (TAN) tka[x] = *reinterpret_cast<const v8bf*>(base + (C::STK * NI + x) * C::TILE + off);
            qq[x] = qf[x][s];
            if constexpr (TAN) tqq[x] = tqf[x][s];
          }
          sacc = mm(ka, qq, sacc);        // S^T = K q^T
          if constexpr (TAN) {
            tacc = mm(ka, tqq, tacc);     // tS^T = K tq^T + tK q^T   (jvp:148-153)
            tacc = mm(tka, qq, tacc);
          }
        }
        float rl = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; ++i) rl = fmaxf(rl, sacc[i]);
        const float rmax = fmaxf(rl, xor32_f(rl));
        // Deferred running max (cdna_hip_programming.md T13; as int8_attn_fwd): the reference moves m
        // to max(m, rowmax) on every tile (jvp:155-158, 164) and rescales l, r, O, A, B by
        // exp2(m - nm).  Here m moves only when some row's tile max exceeds it by more than JVP_THR
        // (log2 units): P = exp2(S qks - m) <= 2^JVP_THR stays in range, and l, r, O, A + B share
        // the same (possibly stale) reference, so O = O/l, tO and lse = m + log2 l are unchanged up
        // to rounding -- while the rescale of the 128 accumulator registers, taken on most tiles of
        // a 32-row wave with the exact rule, becomes rare.
        const float cand = fmaxf(m, rmax * qks);
        if (__ballot(cand > m + JVP_THR)) {
          asm volatile("" ::: "memory");   // keep the rare rescale a branch
          const float rs = exp2_f32(m - cand);
          m = cand;
          l *= rs;
          if constexpr (TAN) racc *= rs;
#pragma unroll
          for (int b = 0; b < C::NDB; ++b) {
            o[b] *= rs;
            if constexpr (TAN) ab[b] *= rs;
          }
        }
        float p[16], hh[16], lt = 0.f, rt = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          p[i] = exp2_f32(sacc[i] * qks - m);      // jvp:160-161
          lt += p[i];
          if constexpr (TAN) {
            hh[i] = p[i] * (tacc[i] * sm);         // jvp:152-153,176
            rt += hh[i];
          }
        }
        lt += xor32_f(lt);
        if constexpr (TAN) rt += xor32_f(rt);
        l += lt;
        if constexpr (TAN) racc += rt;             // jvp:178
        constexpr bool HLO = TAN && !X3 && QA_JVP_HLO;
        v8bf pb[2][NI], hb[2][NI], hlo[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v4u pp[NI], hp[NI], hl;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float p0 = p[8 * s + 2 * j], p1 = p[8 * s + 2 * j + 1];
            const float h0 = hh[8 * s + 2 * j], h1 = hh[8 * s + 2 * j + 1];
            pp[0][j] = pk_bf16(p0, p1);
            if constexpr (TAN) hp[0][j] = pk_bf16(h0, h1);
            if constexpr (HLO)
              hl[j] = pk_bf16(h0 - __uint_as_float(hp[0][j] << 16), h1 - __uint_as_float(hp[0][j] & 0xffff0000u));
            if constexpr (X3) {
              pp[1][j] = pk_bf16(p0 - __uint_as_float(pp[0][j] << 16), p1 - __uint_as_float(pp[0][j] & 0xffff0000u));
              if constexpr (TAN)
                hp[1][j] = pk_bf16(h0 - __uint_as_float(hp[0][j] << 16), h1 - __uint_as_float(hp[0][j] & 0xffff0000u));
            }
          }
#pragma unroll
          for (int x = 0; x < NI; ++x) {
            pb[s][x] = __builtin_bit_cast(v8bf, pp[x]);
            hb[s][x] = __builtin_bit_cast(v8bf, hp[x]);
          }
          if constexpr (HLO) hlo[s] = __builtin_bit_cast(v8bf, hl);
        }
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            v8bf va[NI], tva[NI];
#pragma unroll
            for (int x = 0; x < NI; ++x) {
              va[x] = jtr_frag<D>(base + (C::SV * NI + x) * C::TILE, 32 * u + 16 * s, b, lane);
              if constexpr (TAN) tva[x] = jtr_frag<D>(base + (C::STV * NI + x) * C::TILE, 32 * u + 16 * s, b, lane);
            }
            o[b] = mm(va, pb[s], o[b]);      // jvp:171
            if constexpr (TAN) {
              ab[b] = mm(tva, pb[s], ab[b]); // jvp:173-174
              ab[b] = mm(va, hb[s], ab[b]);  // jvp:180-181
              if constexpr (HLO) ab[b] = mfma_bf16(va[0], hlo[s], ab[b]);
            }
          }
        }


      }
    }
    dma_wait_barrier();
  }
  if (!active) return;
  const long r = (long)bh * Sq + qi;
  if (h == 0) a.lse[r] = m + log2_f32(l);          // jvp:183
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4f wo, wt;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float of = o[b][4 * g + j] / l;                   // jvp:188
        wo[j] = of;
        if constexpr (TAN) wt[j] = (ab[b][4 * g + j] - racc * of) / l;   // jvp:190
      }
      *reinterpret_cast<v4f*>(a.out + r * D + 32 * b + 8 * g + 4 * h) = wo;
      if constexpr (TAN) *reinterpret_cast<v4f*>(a.tout + r * D + 32 * b + 8 * g + 4 * h) = wt;
    }
  }
}

// hi = bf16(x), lo = bf16(x - hi)  (RNE both), n elements, n % 4 == 0
__global__ void split_bf16_kernel(const float* __restrict__ x, __bf16* __restrict__ hi,
                                  __bf16* __restrict__ lo, long n4) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const v4f v = reinterpret_cast<const v4f*>(x)[i];
  const unsigned h01 = pk_bf16(v[0], v[1]), h23 = pk_bf16(v[2], v[3]);
  const unsigned l01 = pk_bf16(v[0] - __uint_as_float(h01 << 16), v[1] - __uint_as_float(h01 & 0xffff0000u));
  const unsigned l23 = pk_bf16(v[2] - __uint_as_float(h23 << 16), v[3] - __uint_as_float(h23 & 0xffff0000u));
  reinterpret_cast<v2u*>(hi)[i] = v2u{h01, h23};
  reinterpret_cast<v2u*>(lo)[i] = v2u{l01, l23};
}

}  // namespace qattn

using namespace qattn;

template <int D, bool X3, bool TAN = true>
static int launch_jvp(const JvpArgs& a, long bh, long sq, hipStream_t st) {
  constexpr int lds = 2 * JvpCfg<D, X3, TAN>::STAGE;
  { static LdsGrant granted_; lds_grant((const void*)jvp_fwd_kernel<D, X3, TAN>, lds, granted_); }
  const int nq = (int)((sq + 127) / 128);
  hipLaunchKernelGGL((jvp_fwd_kernel<D, X3, TAN>), dim3((unsigned)(nq * bh)), dim3(256), lds, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

static JvpArgs jvp_args(const void* const* img, void* out, void* tout, void* lse, long bh, long sq,
                        long sk, int group, float qks, float sm, int nimg) {
  JvpArgs a;
  const __bf16** dst[6] = {a.q, a.k, a.v, a.tq, a.tk, a.tv};
  for (int t = 0; t < 6; ++t) {
    dst[t][0] = (const __bf16*)img[nimg * t];
    dst[t][1] = (const __bf16*)img[nimg * t + nimg - 1];
  }
  a.out = (float*)out;
  a.tout = (float*)tout;
  a.lse = (float*)lse;
  a.BH = (int)bh;
  a.Sq = (int)sq;
  a.Sk = (int)sk;
  a.G = group;
  a.qks = qks;
  a.sm = sm;
  return a;
}

extern "C" int qattn_jvp_fwd_ex(const void* q, const void* k, const void* v, const void* tq,
                                const void* tk, const void* tv, void* out, void* tout, void* lse, long bh,
                                long sq, long sk, int group, int head_dim, float qks, float sm,
                                void* stream) {
  if (sq % 32 != 0 || sk % 64 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq == 0) return 0;
  const void* img[6] = {q, k, v, tq, tk, tv};
  const JvpArgs a = jvp_args(img, out, tout, lse, bh, sq, sk, group, qks, sm, 1);
  hipStream_t st = (hipStream_t)stream;
  return head_dim == 128 ? launch_jvp<128, false>(a, bh, sq, st) : launch_jvp<64, false>(a, bh, sq, st);
}

extern "C" int qattn_jvp_fwd(const void* q, const void* k, const void* v, const void* tq, const void* tk,
                             const void* tv, void* out, void* tout, void* lse, long bh, long sq, long sk,
                             int head_dim, int flags, float qks, float sm, void* stream) {
  if (flags != 0) return 1;
  return qattn_jvp_fwd_ex(q, k, v, tq, tk, tv, out, tout, lse, bh, sq, sk, 1, head_dim, qks, sm, stream);
}

extern "C" int qattn_jvp_fwd_x3_ex(const void* q_hi, const void* q_lo, const void* k_hi, const void* k_lo,
                                   const void* v_hi, const void* v_lo, const void* tq_hi,
                                   const void* tq_lo, const void* tk_hi, const void* tk_lo,
                                   const void* tv_hi, const void* tv_lo, void* out, void* tout, void* lse,
                                   long bh, long sq, long sk, int group, int head_dim, float qks, float sm,
                                   void* stream) {
  if (sq % 32 != 0 || sk % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq == 0) return 0;
  const void* img[12] = {q_hi, q_lo, k_hi, k_lo, v_hi, v_lo, tq_hi, tq_lo, tk_hi, tk_lo, tv_hi, tv_lo};
  const JvpArgs a = jvp_args(img, out, tout, lse, bh, sq, sk, group, qks, sm, 2);
  hipStream_t st = (hipStream_t)stream;
  return head_dim == 128 ? launch_jvp<128, true>(a, bh, sq, st) : launch_jvp<64, true>(a, bh, sq, st);
}

extern "C" int qattn_jvp_fwd_x3(const void* q_hi, const void* q_lo, const void* k_hi, const void* k_lo,
                                const void* v_hi, const void* v_lo, const void* tq_hi, const void* tq_lo,
                                const void* tk_hi, const void* tk_lo, const void* tv_hi, const void* tv_lo,
                                void* out, void* tout, void* lse, long bh, long sq, long sk, int head_dim,
                                float qks, float sm, void* stream) {
  return qattn_jvp_fwd_x3_ex(q_hi, q_lo, k_hi, k_lo, v_hi, v_lo, tq_hi, tq_lo, tk_hi, tk_lo, tv_hi, tv_lo,
                             out, tout, lse, bh, sq, sk, 1, head_dim, qks, sm, stream);
}

// Primal-only launches (O, lse; no tangents): bit-identical O / lse to qattn_jvp_fwd_ex /
// qattn_jvp_fwd_x3_ex on the same primals.
extern "C" int qattn_jvp_primal_ex(const void* q, const void* k, const void* v, void* out, void* lse,
                                   long bh, long sq, long sk, int group, int head_dim, float qks,
                                   float sm, void* stream) {
  if (sq % 32 != 0 || sk % 64 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq == 0) return 0;
  const void* img[6] = {q, k, v, q, k, v};
  const JvpArgs a = jvp_args(img, out, out, lse, bh, sq, sk, group, qks, sm, 1);
  hipStream_t st = (hipStream_t)stream;
  return head_dim == 128 ? launch_jvp<128, false, false>(a, bh, sq, st)
                         : launch_jvp<64, false, false>(a, bh, sq, st);
}

extern "C" int qattn_jvp_primal_x3_ex(const void* q_hi, const void* q_lo, const void* k_hi,
                                      const void* k_lo, const void* v_hi, const void* v_lo, void* out,
                                      void* lse, long bh, long sq, long sk, int group, int head_dim,
                                      float qks, float sm, void* stream) {
  if (sq % 32 != 0 || sk % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq == 0) return 0;
  const void* img[12] = {q_hi, q_lo, k_hi, k_lo, v_hi, v_lo, q_hi, q_lo, k_hi, k_lo, v_hi, v_lo};
  const JvpArgs a = jvp_args(img, out, out, lse, bh, sq, sk, group, qks, sm, 2);
  hipStream_t st = (hipStream_t)stream;
  return head_dim == 128 ? launch_jvp<128, true, false>(a, bh, sq, st)
                         : launch_jvp<64, true, false>(a, bh, sq, st);
}

extern "C" int qattn_split_bf16(const void* x, void* hi, void* lo, long n, void* stream) {
  if (n % 4 != 0) return 1;
  if (n == 0) return 0;
  const long n4 = n / 4;
  hipLaunchKernelGGL(split_bf16_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const float*)x, (__bf16*)hi, (__bf16*)lo, n4);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
