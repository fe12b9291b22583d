// SageAttention-3 int8 attention forward for gfx950 (replaces the attention part of
// helion_atten_int8_hl_dot_fwd, attention_int8.py:170-257), per (batch, head).
//
// Work decomposition
//   * one workgroup = 4 waves = 128 query rows of one (b,h); wave w owns rows 32w..32w+31 = one
//     32-token q-quant block (one sq scale per wave).  2 workgroups per CU (<= 256 VGPRs).
//   * keys stream in 32-key tiles (= one Bkv block) through a 4-slot LDS ring filled by buffer
//     LDS-DMA (no staging registers; the bank swizzle is applied to the per-lane source offset, the
//     LDS image is written lane-linearly).  One barrier per tile; the DMA of tile t+3 is issued
//     right after the barrier of tile t.
//   * per-tile scales of the head sit in LDS (loaded once); workgroups of one head share an XCD.
//
// Per 32-key tile and wave (swapped orientation: keys in registers, query on the lane pair l, l^32),
// software-pipelined by one tile so that each wave has MFMA work beside its softmax VALU:
//     QK(t+1)   S^T = K_i8 . Q_i8^T                   D/32 x v_mfma_i32_32x32x32_i8
//     SM2(t)    e = exp2(d), l, P_i8                  (VALU, beside the QK(t+1) MFMAs)
//     PV(t)     O^T += dequant(V^T . P_i8^T)          D/32 x v_mfma_i32_32x32x32_i8
//     SM1(t+1)  d = S - rowmax, deferred running max  (VALU, beside the PV(t) MFMAs)
// Reference rounding points (int8:197-257):
//     S  = f16(acc * c),  c = sq*sk*qks          on the biased accumulator: one v_pk_fma_f32 per pair
//                                                + v_cvt_pk_f16_f32 (common.h KMAG: no int -> float
//                                                conversion)
//     rm = f16(max_k(acc) * c)                   (c > 0: the row max commutes with the scaling)
//     d  = f16(S - rm)                           (S rounded to f16 first, as the reference does)
//     e  = exp2(d);  P_i8 = trunc(127 e);  sp = exp2(rm - m)/127  (int8:211-237)
//     l += exp2(rm - m) * sum e (fp32);  O *= exp2(m_old - m) when the running max moves.
// Deferred max (cdna_hip_programming.md T13): the running max m moves only when some row's tile max
// exceeds it by more than THR = 8 (log2 units); P_i8 depends only on S - rowmax(tile), O and l share
// the (possibly stale) reference, so O / l is unchanged up to rounding.
//
// Two P_i8 chains.  The fast one above, trunc(127 exp2_f16(f16(S - rm))), equals the reference's
// trunc(exp2(f16(S - m)) / sp) up to the last bits of the f16 exponential, i.e. it moves P_i8 by one
// step now and then.  Such a step weighs sp / l of the row: nothing on a row many keys carry, up to
// |v| / 127 on a row a handful of keys carry (peaked rows).  Tiles that can weigh that much -- some
// row of the wave has er * LIT_K > l, the tile's weight against the row sum so far, and always the
// first tile and the causal diagonal tiles -- take the reference's chain literally instead: S
// rounded in the reference's product order ((X sq) sk) qks, the undeferred running max mt,
// P = exp2(f16(S - mt)) correctly rounded (exp2_cr), sp = f32(exp2(f16(rm - mt)) / 127) and
// P_i8 = trunc(P / sp) with the IEEE quotient.  At config 3 about 2 % of the tiles
// vote literal (tools/fwd_emul.py).
//
// P.V (int8:249-250, O += (P_i8 . v_i8) * sp * sv per 32-key tile): the literal contraction,
// v_mfma_i32_32x32x32_i8 on P_i8 x v_i8 (V^T operand image vt from qattn_int8_quant_vt), exact int32
// per tile, then one fused dequantisation per accumulator element and tile, O += acc * sp*sv (biased
// accumulator: 1 VALU per element instead of 2).  Coarser P.V blocks (one dequantisation per 2 or 4
// tiles) move O by 1.3e-2 .. 6e-2 from the reference (tools/pv_quant_study.py), past the 1e-2 bar.
// (An f16 P.V form on f16(P_i8 sp) x f16(v_i8 sv) measured 10-15 % slower and was removed in round 5.)
#include <climits>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "int8_fwd_plan.h"

namespace qattn {

// (compiles to v_max3_i32).  Deliberately NOT inline asm: its inputs are MFMA results, and hipcc's
// hazard recogniser inserts the MFMA-result -> VALU wait states only for instructions it emits itself.
QA_DEVICE int imax3(int a, int b, int c) { return max(max(a, b), c); }

// Per-wave softmax state between the two halves of a tile.
struct SmTile {
  v2h d[8];       // f16(S - rm) for the 16 scores of this lane (literal tiles: LitOut::d)
  float er;       // exp2(rm - m) (0 on literal tiles: their row sum is in l already)
  float cpv;      // the tile's dequantisation factor sp * sv (in units of the deferred m)
};

// Shapes: BH = batch * query heads, Sq query and Sk key tokens per head; query head
// bh reads key/value head bh / G (grouped-query attention, G = Hq / Hkv).  CAUSAL keeps key <=
// query + qoff: qoff = 0 aligns the first query with the first key (top-left), qoff = Sk - Sq the
// last with the last (bottom-right: new queries against a key/value cache); masked
// scores are excluded (P = 0).  The reference has neither (its int8 path is square, ungrouped and
// non-causal, int8:122-127, 344); these are extensions.
// vt: the V^T operand image (qattn_int8_quant_vt).
// SPLIT (key-split decoding, non-causal): workgroup (x, y) covers keys [y ks, y ks + ks) of
// its query rows and writes the partial state instead of O: through `out`, opart f16
// [split][BH*Sq][D] = f16(O_s / l_s) (the split's normalised output); through `lse`, ml f32x2
// [split][BH*Sq] = {m_s, l_s} (running max, row sum); int8_split_combine_kernel merges the splits.  (The two
// outputs reuse the pointer arguments and ks the causal offset qoff: the causal instantiations are
// at the SGPR limit, one more kernel argument pushes their buffer descriptors into VGPRs.)
// Diagnostic build only (-DQA_FWD_STAMP=1, tools/fwd_stamps.py): s_memrealtime stamps (100 MHz) of
// every workgroup -- entry, end of the prologue, end of the tile loop, exit -- written by lane 0 of
// wave 0 with vector stores to a buffer of their own that no other code reads.
#ifndef QA_FWD_STAMP
#define QA_FWD_STAMP 0
#endif

// QA_FWD_UNROLL (A/B): 0 keeps the run-time-slot loop for every instantiation
#ifndef QA_FWD_UNROLL
#define QA_FWD_UNROLL 1
#endif
// QA_FWD_HG (A/B): causal grid order -- longest-first within groups of this many heads per XCD
// (0: longest-first over all heads)
#ifndef QA_FWD_HG
#define QA_FWD_HG 0
#endif
// QA_FWD_UNROLL_CAUSAL (A/B): the ring-slot unroll in the causal instantiations too (their
// mask-free tiles before the diagonal band)
#ifndef QA_FWD_UNROLL_CAUSAL
#define QA_FWD_UNROLL_CAUSAL 1
#endif
// Timing-only ablations of the ring skeleton (-DQA_FWD_ABL=N, tools/ab_time.py; wrong results):
// 1 no wait+barrier on odd tiles of the unrolled group, 2 also one DMA issue (2 tiles) per 2 tiles,
// 3 no DMA after the prologue, 4 no wait+barrier in the loop
#ifndef QA_FWD_ABL
#define QA_FWD_ABL 0
#endif
// tiles between two foldings of the KMAG bias out of O (rebias in the body; 0 = never)
#ifndef QA_FWD_REBIAS
#define QA_FWD_REBIAS 32
#endif
#ifndef QA_FWD_DQ_SCALAR
#define QA_FWD_DQ_SCALAR 0
#endif
#ifndef QA_FWD_S_SCALAR
#define QA_FWD_S_SCALAR 0
#endif
// Diagnostic build only (-DQA_FWD_LIT_COUNT=1, tools/ab_time.py): counts the literal wave-tiles and
// all wave-tiles (vector atomics by lane 0 of each wave).
#ifndef QA_FWD_LIT_COUNT
#define QA_FWD_LIT_COUNT 0
#endif
#if QA_FWD_LIT_COUNT
__device__ unsigned long long g_fwd_lit[4];   // literal wave-tiles, wave-tiles, marked waves, waves
#endif
#if QA_FWD_STAMP
__device__ unsigned long long g_fwd_stamp[8192][4];
#define FWD_STAMP(k)                                                                            \
  do {                                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < 8192)                                                  \
      g_fwd_stamp[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                            \
  } while (0)
#else
#define FWD_STAMP(k) do { } while (0)
#endif
// The reference's P_i8 chain for one tile (int8:197-237), literally: S in its product order,
// next_m = max(mt, rm) with the undeferred running max, P = exp2(f32(f16(S - next_m))) correctly
// rounded, sp = exp2(f32(f16(rm - next_m))) / 127 (IEEE), P_i8 = trunc(P / sp) with the quotient
// rounded once (through f64: P * RN(1/sp) is within 2^-52 of P / sp, and a quotient of two floats
// that is not a rounding midpoint lies at least 2^-49 from one, so the f32 rounding is the IEEE
// quotient's).  MASK: masked scores (INT_MIN, causal) get P = 0.  acc: the tile's biased S^T
// accumulator, mx its row max; m: the kernel's deferred running max, the unit of the returned row sum
// and dequantisation factor.
// P_i8 leaves as an exponent d = f16(log2(f16(P_i8 / 127 + 0.5 / 127))) that the fast chain's own
// second half turns back into P_i8 = trunc(127 exp2_f16(d)) (exactly: every P_i8 lands at least
// 0.42 from both ends of its unit interval, for any rounding of the f16 log2 within one ulp), so the
// tile loop keeps one SM2 and no second copy of the tile state.
// (S - next_m is one f16 subtraction here where the reference's eager form rounds through f32 first:
// the two differ only when that f32 difference is inexact and lands on an f16 midpoint, which needs an
// odd-integer-spaced difference of operands whose exponents are more than 13 apart -- impossible for
// f16 operands.)
struct LitOut {
  v2h d[8];       // the exponents encoding P_i8
  float er;       // the tile's row sum (this lane's half), in units of m
  float cpv;      // sp * sv, in units of m
  _Float16 mt;    // the running max after the tile
};
QA_DEVICE void log2_pk4(const v2h* x, v2h* r) { QA_PK4("v_log_f16"); }
template <bool MASK>
QA_DEVICE LitOut literal_chain(const v16i& acc, int mx, float cq, float skt, float svt, float qks,
                               _Float16 mt, _Float16 m, LdsI8* tab) {
  LitOut r;
  const float nkq = -KMAG * cq;                  // exact: sq has 11 significant bits
  // fl((X + KMAG) sq - KMAG sq) = fl(X sq) (one rounding), then * sk, * qks (int8:200)
  auto s32 = [&](int a) -> float { return (__builtin_fmaf(__int_as_float(a), cq, nkq) * skt) * qks; };
  const bool kept = !MASK || mx != INT_MIN;     // the row keeps a key of this tile
  const _Float16 rmr = (_Float16)s32(mx);        // (rounding is monotone: the max of the S)
  const _Float16 nmr = (kept && rmr > mt) ? rmr : mt;
  const float sp = kept ? exp2_cr((_Float16)(rmr - nmr), tab) / 127.0f : 0.f;
  const double rsp = sp > 0.f ? 1.0 / (double)sp : 0.0;
  const v2h nm2 = {nmr, nmr};
  const v2h c1 = {(_Float16)(1.0f / 127.0f), (_Float16)(1.0f / 127.0f)};
  const v2h c0 = {(_Float16)(0.5f / 127.0f), (_Float16)(0.5f / 127.0f)};
  float lt = 0.f;
  v2h w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const v2h x = __builtin_bit_cast(v2h, pk_f16(s32(acc[2 * j]), s32(acc[2 * j + 1]))) - nm2;
    v2h pi;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float p = exp2_cr(x[e], tab);
      if (MASK && (acc[2 * j + e] == INT_MIN || !kept)) p = 0.f;
      lt += p;
      pi[e] = (_Float16)__builtin_truncf((float)((double)p * rsp));
    }
    w[j] = __builtin_elementwise_fma(pi, c1, c0);
  }
  log2_pk4(&w[0], &r.d[0]);
  log2_pk4(&w[4], &r.d[4]);
  const float wm = kept ? exp2_f32((float)nmr - (float)m) : 0.f;   // next_m units -> m units
  r.er = lt * wm;
  r.cpv = (sp * svt) * wm;
  r.mt = nmr;
  return r;
}

// QF (quantise q in the prologue, int8:178-186): q16 holds the fp16 queries; each wave quantises its
// own 32-row block -- exactly the Q fragment it needs, one lane (row, half) per 64 values, bit-exact
// with quant_block32_kernel -- and writes q_i8 and sq (the forward's outputs, int8:259-262) and, when
// qbf is not null, the bf16 image of q_i8 the backward reads.  No separate q pass over HBM.
// Deferred votes (DEFER).  The vote asks whether a tile can weigh more than 1/LIT_K of its row; the
// row sum it can compare with is the one so far, but what matters is the FINAL one, and on rows many
// keys carry the tiles that vote -- the first ones, before the sum has grown -- end up weighing
// little (config 3: ~1.5 % of the tiles vote, ~4 % of the kernel's time if they took the literal
// chain).  So the forward takes the fast chain on every tile and only writes down each vote -- the
// tile's weight er and the running max m at the time, in LDS (no register is free across the loop),
// NV slots per wave -- and at the end takes the votes again against the final row sums, each
// weight rescaled by exp2(m_then - m).  A wave for which one still holds (or whose slots overflowed)
// marks its rows with FIX_LSE16 (lse; FIX_M32: m of the split state), and the fixup launch (FIX: the
// same kernel, voting at the tile, the literal chain where a vote holds) recomputes exactly those
// waves and overwrites their O and lse; its workgroups without a marked wave exit at once.
constexpr unsigned short FIX_LSE16 = 0x7e5au;    // an fp16 NaN no result carries
constexpr unsigned FIX_M32 = 0x7fc0e5a5u;        // an fp32 NaN no result carries

// The kernel body.  INL (the inline fixup): the marks travel through mark_lds, WAVES words in LDS,
// instead of the lse sentinel; the fast pass and the fixup pass run in one workgroup (see
// int8_attn_fwd_kernel).
template <int D, bool CAUSAL, bool SPLIT, bool QF, bool FIX, bool INL>
QA_DEVICE __attribute__((always_inline)) void int8_attn_fwd_body(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const int8_t* __restrict__ vt, const _Float16* __restrict__ sv,
    _Float16* __restrict__ out, _Float16* __restrict__ lse, int BH, int Sq, int Sk, int G, int qoff,
    float qks, const _Float16* __restrict__ q16, __bf16* __restrict__ qbf, unsigned* mark_lds) {
  static_assert(!SPLIT || !CAUSAL, "key splits: non-causal");
  static_assert(!SPLIT || !QF, "key splits: pre-quantised q");
  static_assert(!FIX || !QF || INL, "the separate fixup reads the q_i8 the forward wrote");
  static_assert(!INL || !SPLIT, "the inline fixup: the non-split forward");
  using C = Int8FwdCfg<D>;
  constexpr bool DEFER = C::LIT_K > 0 && QA_FWD_DEFER > 0 && !FIX;
  FWD_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per-tile scales: ck = sk * qks (f32), sv / 127 (f32)
  float* ck_lds = reinterpret_cast<float*>(smem + C::RING);

  const int nq = (Sq + C::QROWS - 1) / C::QROWS;
  int bh, qt;
  if constexpr (CAUSAL && QA_FWD_HG > 0) xcd_remap_lpt_grouped(blockIdx.x, nq, BH, true, QA_FWD_HG, bh, qt);
  else if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nq, BH, true, bh, qt);
  else xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int q0 = qt * C::QROWS + wave * 32;
  bool active = q0 < Sq;
  const long head_row0 = (long)bh * Sq;           // this head's query rows
  const int split = SPLIT ? (int)__builtin_amdgcn_readfirstlane(blockIdx.y) : 0;
  if constexpr (FIX) {   // the waves the forward marked; a workgroup without one exits at once
    bool any = false;
#pragma unroll
    for (int w = 0; w < C::WAVES; ++w) {
      const int r0 = qt * C::QROWS + w * 32;
      bool f = false;
      if (r0 < Sq) {
        if constexpr (INL)
          f = mark_lds[w] != 0;
        else if constexpr (SPLIT)
          f = __float_as_uint(reinterpret_cast<const float2*>(lse)[((long)split * BH + bh) * Sq + r0].x) ==
              FIX_M32;
        else
          f = __builtin_bit_cast(unsigned short, lse[head_row0 + r0]) == FIX_LSE16;
      }
      any = any || f;
      if (w == wave) active = active && f;
    }
    if (!any) return;
  }
  const int ks = qoff;                             // SPLIT (non-causal): keys per split
  const int k0 = SPLIT ? split * ks : 0;           // first key of this workgroup's key range
  const int nk = SPLIT ? min(ks, Sk - k0) : Sk;    // its keys
  const long kv_row0 = (long)(bh / G) * Sk + k0;  // its key/value head's rows
  const int8_t* kbase = k_i8 + kv_row0 * D;
  const int8_t* vbase = vt + kv_row0 * D;
  // causal: key tiles past the workgroup's last query are masked for all of its rows
  const int nt = CAUSAL ? min(Sk / C::KT, (qt * C::QROWS + C::QROWS + qoff + C::KT - 1) / C::KT)
                        : nk / C::KT;
  // per-tile scales, shifted by one tile: entry i holds tile min(i + 1, nt - 1), the tile whose SM1
  // runs in loop iteration i, so that 4 iterations read their scales with one 16-B LDS read
  float* svq_lds = ck_lds + ((nt + 3) & ~3);
  // the exp2 correction table of the literal chain (exp2_corr.h), after the scale tables; in the
  // fast pass (DEFER) the same region holds the deferred votes instead (the table is not loaded)
  unsigned* corr_lds = reinterpret_cast<unsigned*>(svq_lds + ((nt + 3) & ~3));

  DmaPlan<D> dma;
  dma.init(wave, lane, Sk - k0, kbase, vbase);   // (the range bound only: reads stay in nk)
  const unsigned smem_lds = lds_addr(smem);
  dma.issue(smem_lds, 0);
  dma.issue(smem_lds + 1 * C::SLOT, min(1, nt - 1));
  dma.issue(smem_lds + 2 * C::SLOT, min(2, nt - 1));
  for (int i = tid; i < nt; i += 64 * C::WAVES) {
    const int ti = min(i + 1, nt - 1);
    ck_lds[i] = (float)sk[kv_row0 / 32 + ti] * qks;
    svq_lds[i] = (float)sv[kv_row0 / 32 + ti] * (1.0f / 127.0f);
  }
  if constexpr (!DEFER)   // (the forward with deferred votes never runs the literal chain)
    for (int i = tid; i < EXP2_CORR_WORDS; i += 64 * C::WAVES) corr_lds[i] = g_exp2_corr[i];
  const float ck0 = (float)sk[kv_row0 / 32] * qks;   // tile 0 (the prologue's SM1)
  const float svq0 = (float)sv[kv_row0 / 32] * (1.0f / 127.0f);

  // ---- Q fragment (B operand of S^T = K Q^T): lane holds Q[q0+c32][32s + 16h .. +16]
  v4i qf[C::NKS];
  float cq = 0.f;
  if (active && QF) {   // quantise the wave's 32-row block (int8:178-186)
    const long row = head_row0 + q0 + c32;
    const _Float16* x16 = q16 + row * D + 16 * h;
    v8h x[C::NKS][2];
    float amax = 0.f;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        x[s][u] = *reinterpret_cast<const v8h*>(x16 + 32 * s + 8 * u);
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf((float)x[s][u][j]));
      }
    amax = wave_max_f(amax);
    const _Float16 s16 = (_Float16)(amax / 127.0f);
    cq = (float)s16;
    const float r = quant_rcp(cq);
    if (lane == 0) const_cast<_Float16*>(sq)[(head_row0 + q0) / 32] = s16;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
      unsigned w[4];
      float qv[16];
      quant8(x[s][0], cq, r, w[0], w[1], qv);
      quant8(x[s][1], cq, r, w[2], w[3], qv + 8);
      qf[s] = v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
      *reinterpret_cast<v4i*>(const_cast<int8_t*>(q_i8) + row * D + 32 * s + 16 * h) = qf[s];
      if (qbf != nullptr) {
        __bf16* ib = qbf + row * D + 32 * s + 16 * h;
#pragma unroll
        for (int u = 0; u < 2; ++u)
          *reinterpret_cast<v4u*>(ib + 8 * u) =
              v4u{pk_bf16(qv[8 * u], qv[8 * u + 1]), pk_bf16(qv[8 * u + 2], qv[8 * u + 3]),
                  pk_bf16(qv[8 * u + 4], qv[8 * u + 5]), pk_bf16(qv[8 * u + 6], qv[8 * u + 7])};
      }
    }
  } else if (active) {
    const int8_t* qrow = q_i8 + (head_row0 + q0 + c32) * D + 16 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v4i*>(qrow + 32 * s);
    cq = (float)sq[(head_row0 + q0) / 32];
  }
  // the biased accumulator seed, opaque to the compiler (so it stays in 16 registers instead of
  // being re-materialised by 16 v_mov per use)
  v16i kmag;
#pragma unroll
  for (int i = 0; i < 16; ++i) kmag[i] = KMAG_BITS;
  asm volatile("" : "+v"(kmag));

  // lane-constant LDS byte offsets: K A-operand chunk (2s+h) of key row c32; piece b of the vt
  // image, 16 B per lane
  int koff[C::NKS], voff[C::NDB];
#pragma unroll
  for (int s = 0; s < C::NKS; ++s) koff[s] = c32 * D + 16 * ((2 * s + h) ^ k_sw<D>(c32));
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) voff[b] = C::K_BYTES + b * 1024 + 16 * lane;

  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  _Float16 m = (_Float16)(-INFINITY);
  // f16(m + THR): the deferred running max moves when a row's tile max exceeds it.  (The f16 sum can
  // round up, so a tile max equal to that rounded value leaves m in place where an fp32 compare would
  // move it: er = exp2(rm - m) then exceeds 2^THR by at most half an f16 ulp of m + THR.  er only
  // scales l and the P.V factor -- P itself is taken against the tile max -- so O and lse stay within
  // rounding of each other either way, but bits can differ from an fp32-compare build.)
  _Float16 m_thr = (_Float16)(-INFINITY);
  _Float16 mt = (_Float16)(-INFINITY);      // the reference's (undeferred) running max
  float l = 0.f;      // per-lane partial (this lane's key half); the reference's l = 1 is wiped by r = 0
  float obias = 0.f;  // sum of the tile dequantisation factors (the KMAG bias of O is KMAG * obias)
  // the dequantisation factor of the tile whose P.V is in flight while SM1 of the next tile runs;
  // a running-max move there rescales it with O (its int32 product is added after SM1)
  float cpv_pend = 0.f;
  int nvote = 0;            // (DEFER) votes written down so far (NV slots; more mark the wave)

  // ring slot u (the loop below passes compile-time slot numbers: LDS offsets become immediates)
  auto slot_at = [&](int u) -> const char* { return smem + u * C::SLOT; };

  // S^T of the tile in ring slot u into a biased int32 accumulator: fragment loads and MFMAs
  // separately, so the K loads of tile t+1 can be issued ahead of the V-operand loads of tile t
  auto qk_load = [&](int u, v4i* kf) {
    const char* kl = slot_at(u);
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) kf[s] = *reinterpret_cast<const v4i*>(kl + koff[s]);
  };
  auto qk_mma = [&](const v4i* kf) -> v16i {
    v16i acc = mfma_i8(kf[0], qf[0], kmag);
#pragma unroll
    for (int s = 1; s < C::NKS; ++s) acc = mfma_i8(kf[s], qf[s], acc);
    return acc;
  };

  // O^T += V^T P^T for tile t: operand loads (issued early, consumed after QK(t+1) and SM2(t))
  // and the MFMAs
  auto pv_load = [&](int u, v4i* va) {
    const char* vl = slot_at(u);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) va[b] = *reinterpret_cast<const v4i*>(vl + voff[b]);
  };
  v16i pacc[C::NDB];
  auto pv_mma = [&](const v4i* va, const v4u* pw) {
    const v4i p = __builtin_bit_cast(v4i, pw[0]);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) pacc[b] = mfma_i8(va[b], p, kmag);
  };
  // O += (KMAG + X) * (sp * sv) for the tile's exact int32 X (one fused op per element)
  auto pv_dequant = [&](float cpv) {
    // explicit v_pk_fma_f32 pairs (scalar v_fma_f32 measured 2-3 % slower);
    // QA_FWD_DQ_SCALAR (A/B, needs -fno-slp-vectorize): the first that many d blocks scalar
    const v2f_ c2 = {cpv, cpv};
#pragma unroll
    for (int b = 0; b < C::NDB; ++b)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        if (b < QA_FWD_DQ_SCALAR) {
          o[b][r] = __builtin_fmaf(__int_as_float(pacc[b][r]), cpv, o[b][r]);
          o[b][r + 1] = __builtin_fmaf(__int_as_float(pacc[b][r + 1]), cpv, o[b][r + 1]);
          continue;
        }
        const v2f_ a = {__int_as_float(pacc[b][r]), __int_as_float(pacc[b][r + 1])};
        const v2f_ y = __builtin_elementwise_fma(a, c2, v2f_{o[b][r], o[b][r + 1]});
        o[b][r] = y[0];
        o[b][r + 1] = y[1];
      }
    obias += cpv;
  };
  // Fold the KMAG bias out of O every QA_FWD_REBIAS tiles: O holds sum_t (KMAG + X_t) c_t, whose
  // magnitude grows with the tiles while the signal sum_t X_t c_t does not, so without it the fp32
  // rounding of the accumulator (correlated from tile to tile: the same c_t) eats the signal on long
  // key ranges (relL2 0.16 against exact attention at 128k keys).  O - KMAG * obias in one fma per
  // element (the product exact inside it); then obias restarts from 0.
  auto rebias = [&]() {
    const v2f_ nk = {-KMAG, -KMAG}, ob = {obias, obias};
#pragma unroll
    for (int b = 0; b < C::NDB; ++b)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const v2f_ y = __builtin_elementwise_fma(nk, ob, v2f_{o[b][r], o[b][r + 1]});
        o[b][r] = y[0];
        o[b][r + 1] = y[1];
      }
    obias = 0.f;
  };

  // first half of the softmax of tile t: row max, d = f16(S - rm), deferred running max, er, the
  // tile's P.V scale, and the literal-chain vote
  //   dg (std::true_type / false_type): whether tile t may cross the diagonal (causal), i.e.
  //   whether the masks are compiled in
  //   pend (std::true_type / false_type): a P.V product is in flight (every SM1 but the prologue's);
  //   the literal branch adds it to O first, which frees its 64 accumulator registers
  auto sm1 = [&](const v16i& acc_in, int t, bool live, SmTile& st, float ckt, float svqt, auto dg,
                 auto pend) {
    // causal tiles crossing this wave's diagonal: keys above the row's query drop out of the max
    // (INT_MIN) and get d = -inf below, so P = 0 and the tile scale ignores them
    const bool diag = CAUSAL && decltype(dg)::value && (t * C::KT + C::KT - 1 > q0 + qoff);
    v16i acc = acc_in;
    if (diag) {
      // key > query as one compare per score against an immediate:
      // t KT + (r & 3) + 8 (r >> 2) + 4h > q0 + qoff + c32  <=>  dd > -((r & 3) + 8 (r >> 2))
      const int dd = t * C::KT + 4 * h - (q0 + qoff + c32);
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (dd > -((r & 3) + 8 * (r >> 2))) acc[r] = INT_MIN;
    }
    int mx = imax3(acc[0], acc[1], acc[2]);
    mx = imax3(mx, acc[3], acc[4]);
    mx = imax3(mx, acc[5], acc[6]);
    mx = imax3(mx, acc[7], acc[8]);
    mx = imax3(mx, acc[9], acc[10]);
    mx = imax3(mx, acc[11], acc[12]);
    mx = imax3(mx, acc[13], acc[14]);
    mx = max(mx, acc[15]);
    {
      auto r = __builtin_amdgcn_permlane32_swap((unsigned)mx, (unsigned)mx, false, false);
      mx = max((int)r[0], (int)r[1]);
    }
    // S = f16(X * c) (int8:200-203: fp32 products, then fp16), on the biased accumulator
    v2h s2[8];
    const float c = kmag_scale(cq * ckt);
    const float nb = -KMAG * c;
    const _Float16 rm = biased_to_f16(mx, c, nb);
    biased_to_f16x16(acc, c, nb, s2);
#if QA_FWD_S_SCALAR > 0   // (A/B, needs -fno-slp-vectorize: the first pairs in scalar fp32)
#pragma unroll
    for (int j = 0; j < QA_FWD_S_SCALAR; ++j)
      s2[j] = v2h{(_Float16)__builtin_fmaf(__int_as_float(acc[2 * j]), c, nb),
                  (_Float16)__builtin_fmaf(__int_as_float(acc[2 * j + 1]), c, nb)};
#endif
    const v2h rm2 = {rm, rm};
#pragma unroll
    for (int j = 0; j < 8; ++j) st.d[j] = s2[j] - rm2;   // f16(S - rm)  (int8:211, 232-236)
    if (diag) {
      const _Float16 ninf = (_Float16)(-INFINITY);
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          if (acc[2 * j + e] == INT_MIN) st.d[j][e] = ninf;
    }
    if (__ballot(rm > m_thr) != 0) {
      // (the empty volatile asm keeps this rare branch a branch: if-converted, the O rescale costs
      // 2 * D / 2 packed multiplies on every tile)
      asm volatile("" ::: "memory");
      const _Float16 nm = m > rm ? m : rm;
      const float r = exp2_f32((float)(_Float16)(m - nm));
      m = nm;
      m_thr = m + (_Float16)C::THR;
      l *= r;
      obias *= r;
      cpv_pend *= r;
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) o[b] *= r;
    }
    st.er = exp2_f32((float)(_Float16)(rm - m));
    st.cpv = st.er * svqt;
    // the vote: the tile can weigh more than 1/LIT_K of the row sum so far (l is this lane's half
    // of it); the first tile (l = 0) always votes.  Causal diagonal tiles always take the chain.
    // (`live` is false for the duplicate tile of the loop's last iteration, whose state is never
    // consumed: the chain adds its row sum to l directly.)
    bool lit = diag;
    if constexpr (C::LIT_K > 0) lit = lit || __ballot(st.er * (0.5f * C::LIT_K) > l) != 0;
    if constexpr (C::LIT_K == 0) lit = true;
    lit = lit && live;
#if defined(QA_FWD_LIT_LOOP) && QA_FWD_LIT_LOOP == 0   // (A/B: votes only in the prologue's tile 0)
    lit = lit && (diag || !decltype(pend)::value);
#endif
#ifdef QA_FWD_LIT_NEVER   // (A/B: the vote and the chain's code, never taken)
    lit = lit && qks < 0.f;
#endif
#if QA_FWD_LIT_COUNT
    if (lane == 0 && live) {
      atomicAdd(&g_fwd_lit[1], 1ull);
      if (lit) atomicAdd(&g_fwd_lit[0], 1ull);
    }
#endif
    if (DEFER && lit) {   // write the vote down (a wave-uniform branch); the tile stays fast
      if (nvote < C::NV) {
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        unsigned* cs = corr_lds + (wave * C::NV + nvote) * 128 + ln;   // (over the unloaded table)
        cs[0] = __float_as_uint(st.er);
        cs[64] = (unsigned)__builtin_bit_cast(unsigned short, m);
      }
      ++nvote;
      lit = false;
    }
    if (lit) {
      asm volatile("" ::: "memory");
      if constexpr (decltype(pend)::value) {
        pv_dequant(cpv_pend);
        cpv_pend = 0.f;   // (the loop's own dequantisation then adds (KMAG + X) * 0)
      }
      const LitOut r = literal_chain<CAUSAL>(acc, mx, cq, (float)sk[kv_row0 / 32 + t],
                                             (float)sv[kv_row0 / 32 + t], qks, mt, m, (LdsI8*)corr_lds);
#pragma unroll
      for (int j = 0; j < 8; ++j) st.d[j] = r.d[j];
      l += r.er;
      st.er = 0.f;
      st.cpv = r.cpv;
      mt = r.mt;
    } else if (!DEFER && mx != INT_MIN && rm > mt) {   // (only the literal chain reads mt)
      mt = rm;
    }
  };

  // second half: e = exp2(d) (sm2_exp), then l += er * sum e and the 16 P_i8 bytes (sm2)
  auto sm2_exp = [&](const SmTile& st, v2h* e) {
    exp2_pk4(&st.d[0], &e[0]);
    exp2_pk4(&st.d[4], &e[4]);
  };
  auto sm2 = [&](const SmTile& st, const v2h* e, v4u* pw) {
    // row sum of e: packed f16 adds (pairs, then sums of 4 and 8 values <= 8), one f32 mix-add
    const v2h s = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
    l = fmaf(pk_hsum(s), st.er, l);
    const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
    unsigned y[8];
    p_index8(e, k127, y);
    pw[0] = __builtin_bit_cast(v4u, pack_p_index(y));
  };

  vmem_drain();
  __syncthreads();
  FWD_STAMP(1);

  SmTile st;
  // One loop iteration per tile t: SM2 and P.V of tile t, QK and SM1 of tile t+1.  The last iteration
  // computes QK / SM1 of a duplicate of the last tile (its slot holds a clamped re-load): harmless
  // (its row max cannot move m, and its state is never used) and it keeps the loop body branch-free.
  //   cur, nxt: ring slots of tiles t and t+1; fill: the slot the DMA of tile t+3 goes to (freed by
  //   the barrier); ckn, svqn: the scales of tile t+1
  auto iter = [&](int t, int cur, int nxt, int fill, float ckn, float svqn, auto dg, int pos) {
#if QA_FWD_ABL   // (timing-only ablations of the ring skeleton: results are wrong)
    const int P = pos;   // (a constant at every call site: 0..3 in the unrolled group, -2 elsewhere)
    if (QA_FWD_ABL == 4 || ((QA_FWD_ABL == 1 || QA_FWD_ABL == 2) && (P & 1))) {
    } else {
      ring_wait_barrier<C::IPW>();
    }
    if (QA_FWD_ABL == 3 || (QA_FWD_ABL == 2 && (P & 1))) {
    } else {
      dma.issue(smem_lds + fill * C::SLOT, min(t + 3, nt - 1));
      if (QA_FWD_ABL == 2 && P >= 0) dma.issue(smem_lds + ((fill + 1) & 3) * C::SLOT, min(t + 4, nt - 1));
    }
#else
    ring_wait_barrier<C::IPW>();   // tile t+1 landed (t+2 may be in flight); slot `fill` is free
    dma.issue(smem_lds + fill * C::SLOT, min(t + 3, nt - 1));
#endif
    // Phase order (pinned: hipcc otherwise issues the QK(t+1) chain right before its consumer
    // SM1(t+1) and the wave stalls on it): fragment reads, the 16 exponentials of tile t (which
    // cover the LDS latency), QK(t+1), then the rest of SM2(t), PV(t) and SM1(t+1).
    const int tn = min(t + 1, nt - 1);
    v4i kf[C::NKS];
    qk_load(nxt, kf);
    v4i va[C::NDB];
    pv_load(cur, va);
    v2h e[8];
    sm2_exp(st, e);
    __builtin_amdgcn_sched_barrier(0);
    const v16i nacc = qk_mma(kf);
    __builtin_amdgcn_sched_barrier(0);
    v4u pw[1];
    sm2(st, e, pw);
    cpv_pend = st.cpv;
    pv_mma(va, pw);
    sm1(nacc, tn, t + 1 < nt, st, ckn, svqn, dg, std::true_type{});   // (may rescale O, obias, cpv_pend)
    pv_dequant(cpv_pend);   // after SM1(t+1), so the PV MFMAs of tile t have retired
  };
  if (active) {
    {
      v4i kf[C::NKS];
      qk_load(0, kf);
      sm1(qk_mma(kf), 0, true, st, ck0, svq0, std::true_type{}, std::false_type{});
    }
    // Causal: iteration t runs SM1 of tile t+1, and tiles below td0 = (first query of the workgroup
    // + qoff) / KT cross no wave's diagonal, so iterations t < td0 - 1 run with the masks compiled
    // out (the same values: nothing is masked there) and the rest, at most WAVES + 1 of them, with
    // them.
    const int tmain = CAUSAL ? max(0, min(nt, (qt * C::QROWS + qoff) / C::KT - 1)) : nt;
    // groups of NSLOT = 4 tiles with compile-time ring slots (immediate LDS offsets, one 16-B read
    // of each scale table per group), then the remaining tiles with run-time slots
    static_assert(C::NSLOT == 4, "ring of 4 slots");
    constexpr bool UNROLL = QA_FWD_UNROLL && (!CAUSAL || QA_FWD_UNROLL_CAUSAL) && (QF || FIX || SPLIT);
    const std::false_type nodiag{};
    int t = 0;
    for (; UNROLL && t + 4 <= tmain; t += 4) {
      const v4f ck4 = *reinterpret_cast<const v4f*>(ck_lds + t);
      const v4f sv4 = *reinterpret_cast<const v4f*>(svq_lds + t);
      iter(t, 0, 1, 3, ck4[0], sv4[0], nodiag, 0);
      iter(t + 1, 1, 2, 0, ck4[1], sv4[1], nodiag, 1);
      iter(t + 2, 2, 3, 1, ck4[2], sv4[2], nodiag, 2);
      iter(t + 3, 3, 0, 2, ck4[3], sv4[3], nodiag, 3);
      if (QA_FWD_REBIAS > 0 && ((t + 4) % QA_FWD_REBIAS) == 0) rebias();
    }
    for (; t < tmain; ++t) {
      iter(t, t & 3, (t + 1) & 3, (t + 3) & 3, ck_lds[t], svq_lds[t], nodiag, -2);
      if (QA_FWD_REBIAS > 0 && ((t + 1) % QA_FWD_REBIAS) == 0) rebias();
    }
    if constexpr (CAUSAL) {
      for (; t < nt; ++t) {
        iter(t, t & 3, (t + 1) & 3, (t + 3) & 3, ck_lds[t], svq_lds[t], std::true_type{},
             -2);
        if (QA_FWD_REBIAS > 0 && ((t + 1) % QA_FWD_REBIAS) == 0) rebias();
      }
    }
  } else {   // a wave past the last query row: the barriers and the ring's DMA only
    for (int t = 0; t < nt; ++t) {
      ring_wait_barrier<C::IPW>();
      dma.issue(smem_lds + ((t + 3) & 3) * C::SLOT, min(t + 3, nt - 1));
    }
  }
  vmcnt_wait_all();
  __syncthreads();   // every wave is done with the ring: its slots become the output staging area
  FWD_STAMP(2);

  if (!active) return;
  // (DEFER) the votes against the final row sums: mark the wave for the fixup
  bool fix = false;
  if (DEFER && nvote > 0) {
    const float lrow = pair_sum(l) * (1.0f / (float)C::LIT_K);
    if (nvote > C::NV) {
      fix = true;
    } else {
      const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
      const unsigned* cs = corr_lds + wave * C::NV * 128 + ln;
      bool any = false;
#pragma unroll
      for (int c = 0; c < C::NV; ++c) {
        if (c >= nvote) break;
        const float w = __uint_as_float(cs[128 * c]) *
                        exp2_f32((float)__builtin_bit_cast(_Float16, (unsigned short)cs[128 * c + 64]) - (float)m);
        any = any || w > lrow;
      }
      fix = __ballot(any) != 0;
    }
  }
#if QA_FWD_LIT_COUNT
  if (DEFER && lane == 0) {
    atomicAdd(&g_fwd_lit[3], 1ull);
    if (fix) atomicAdd(&g_fwd_lit[2], 1ull);
  }
#endif
  if constexpr (SPLIT) {   // the partial state of this key range: {m, l} and f16(O / l)
    l = pair_sum(l);
    const long prow = ((long)split * BH + bh) * Sq + q0;
    if (h == 0)
      reinterpret_cast<float2*>(lse)[prow + c32] = float2{fix ? __uint_as_float(FIX_M32) : (float)m, l};
    const float inv = 1.0f / l;
    store_rows<D, _Float16, 1, true>(o, inv, smem + wave * RowTile<D, _Float16>::BYTES,
                                     out + prow * D, lane, -KMAG * obias * inv);
    return;
  }
  // ---------------- epilogue: lse = fp16(m + fp16(log2 l)); O = fp16(O / l)   (int8:252-257)
  l = pair_sum(l);
  const long qrow = head_row0 + q0 + c32;
  if (INL && fix && lane == 0) mark_lds[wave] = 1u;
  if (h == 0)
    lse[qrow] = (fix && !INL) ? __builtin_bit_cast(_Float16, FIX_LSE16)
                              : (_Float16)((float)m + (float)(_Float16)log2_f32(l));
  const float inv = 1.0f / l;
  store_rows<D, _Float16, 1, true>(o, inv, smem + wave * RowTile<D, _Float16>::BYTES,
                                   out + (head_row0 + q0) * D, lane, -KMAG * obias * inv);
#if QA_FWD_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  FWD_STAMP(3);
#endif
}

// QA_FWD_INLINE_FIX (A/B): the non-split forward redoes its marked waves in the same workgroup, right
// after the fast pass (a second, literal-chain pass over the tiles, with q quantised again from q16),
// instead of in a second launch
#ifndef QA_FWD_INLINE_FIX
#define QA_FWD_INLINE_FIX 1
#endif
template <int D, bool CAUSAL, bool SPLIT = false, bool QF = false, bool FIX = false, bool INL = false>
__global__ __launch_bounds__((64 * Int8FwdCfg<D>::WAVES), 2) void int8_attn_fwd_kernel(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const int8_t* __restrict__ vt, const _Float16* __restrict__ sv,
    _Float16* __restrict__ out, _Float16* __restrict__ lse, int BH, int Sq, int Sk, int G, int qoff,
    float qks, const _Float16* __restrict__ q16, __bf16* __restrict__ qbf) {
  if constexpr (!INL) {
    int8_attn_fwd_body<D, CAUSAL, SPLIT, QF, FIX, false>(q_i8, sq, k_i8, sk, vt, sv, out, lse, BH, Sq, Sk, G,
                                                         qoff, qks, q16, qbf, nullptr);
  } else {
    using C = Int8FwdCfg<D>;
    extern __shared__ __attribute__((aligned(16))) char smem_k[];
    // after the body's LDS regions for any workgroup (sized for all key tiles)
    unsigned* marks = reinterpret_cast<unsigned*>(smem_k + C::lds_bytes(Sk / C::KT));
    if (threadIdx.x < C::WAVES) marks[threadIdx.x] = 0u;   // (published by the body's first barrier)
    int8_attn_fwd_body<D, CAUSAL, false, QF, false, true>(q_i8, sq, k_i8, sk, vt, sv, out, lse, BH, Sq, Sk,
                                                          G, qoff, qks, q16, qbf, marks);
    __syncthreads();
    bool any = false;
#pragma unroll
    for (int w = 0; w < C::WAVES; ++w) any = any || marks[w] != 0u;
    if (any)
      int8_attn_fwd_body<D, CAUSAL, false, QF, true, true>(q_i8, sq, k_i8, sk, vt, sv, out, lse, BH, Sq, Sk,
                                                           G, qoff, qks, q16, qbf, marks);
  }
}

// Diagnostic switch (tests/test_gpu_fixup.py): QATTN_FWD_SKIP_FIXUP=1 leaves out the separate fixup
// launches, so the marks of the waves the fast pass handed over stay in lse (FIX_LSE16) / ml
// (FIX_M32) where a test can count them.  Read per call; never set in production.
static bool skip_fixup() {
  const char* e = std::getenv("QATTN_FWD_SKIP_FIXUP");
  return e != nullptr && e[0] == '1';
}

template <int D, bool CAUSAL, bool QF>
static int launch_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                      const void* vt, const void* sv, void* out, void* lse, long bh, long sq_tok,
                      long sk_tok, int group, int qoff, float qks, const void* q16, void* qbf,
                      hipStream_t st) {
  using C = Int8FwdCfg<D>;
  const int nq = (int)((sq_tok + C::QROWS - 1) / C::QROWS);
  const int lds = C::lds_bytes((int)(sk_tok / 32));
  // the inline fixup (q quantised in the kernel: the fixup pass quantises it again from q16)
  constexpr bool INL = QA_FWD_INLINE_FIX && QF && C::LIT_K > 0 && QA_FWD_DEFER;
  auto kern = int8_attn_fwd_kernel<D, CAUSAL, false, QF, false, INL>;
  const int lds_k = lds + (INL ? 4 * C::WAVES : 0);
  { static LdsGrant granted_; if (!lds_grant((const void*)kern, lds_k, granted_)) return 1; }
  hipLaunchKernelGGL(kern, dim3((unsigned)(nq * bh)), dim3(64 * C::WAVES), lds_k, st,
                     (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,
                     (const int8_t*)vt, (const _Float16*)sv, (_Float16*)out, (_Float16*)lse, (int)bh,
                     (int)sq_tok, (int)sk_tok, group, qoff, qks, (const _Float16*)q16, (__bf16*)qbf);
  if constexpr (C::LIT_K > 0 && QA_FWD_DEFER && !INL) {   // the waves whose votes held: redone
    if (skip_fixup()) return hipGetLastError() == hipSuccess ? 0 : 2;
    auto fixk = int8_attn_fwd_kernel<D, CAUSAL, false, false, true>;
    { static LdsGrant granted_; if (!lds_grant((const void*)fixk, lds, granted_)) return 1; }
    hipLaunchKernelGGL(fixk, dim3((unsigned)(nq * bh)), dim3(64 * C::WAVES), lds, st,
                       (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,
                       (const int8_t*)vt, (const _Float16*)sv, (_Float16*)out, (_Float16*)lse, (int)bh,
                       (int)sq_tok, (int)sk_tok, group, qoff, qks, nullptr, nullptr);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Merge of the key splits (flash-decoding): per row M = max_s m_s, w_s = exp2(m_s - M) l_s,
// L = sum_s w_s, O = f16(sum_s w_s Ô_s / L) with Ô_s = O_s / l_s the split's normalised output,
// lse = f16(M + f16(log2 L)) (int8:252-257 on the merged state).  One thread per 8 columns of a row.
template <int D>
__global__ __launch_bounds__(256) void int8_split_combine_kernel(const _Float16* __restrict__ opart,
                                                                 const float2* __restrict__ ml,
                                                                 _Float16* __restrict__ out,
                                                                 _Float16* __restrict__ lse, long rows,
                                                                 int nsplit) {
  constexpr int TPR = D / 8;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long row = gid / TPR;
  const int c = (int)(gid % TPR);
  if (row >= rows) return;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[s * rows + row].x);
  float L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nsplit; ++s) {
    const float2 v = ml[s * rows + row];
    const float w = exp2_f32(v.x - M) * v.y;
    L += w;
    const v8h a = *reinterpret_cast<const v8h*>(opart + ((long)s * rows + row) * D + 8 * c);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = fmaf(w, (float)a[i], acc[i]);
  }
  const float inv = 1.0f / L;
  v8h o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (_Float16)(acc[i] * inv);
  *reinterpret_cast<v8h*>(out + row * D + 8 * c) = o;
  if (c == 0) lse[row] = (_Float16)(M + (float)(_Float16)log2_f32(L));
}

template <int D>
static int launch_fwd_split(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                            const void* vt, const void* sv, void* opart, void* ml, long bh, long sq_tok,
                            long sk_tok, int group, int ks, float qks, hipStream_t st) {
  using C = Int8FwdCfg<D>;
  const int nq = (int)((sq_tok + C::QROWS - 1) / C::QROWS);
  const int nsplit = (int)((sk_tok + ks - 1) / ks);
  const int lds = C::lds_bytes(ks / 32);
  { static LdsGrant granted_; if (!lds_grant((const void*)int8_attn_fwd_kernel<D, false, true>, lds, granted_)) return 1; }
  hipLaunchKernelGGL((int8_attn_fwd_kernel<D, false, true>), dim3((unsigned)(nq * bh), (unsigned)nsplit),
                     dim3(64 * C::WAVES), lds, st, (const int8_t*)q_i8, (const _Float16*)sq,
                     (const int8_t*)k_i8, (const _Float16*)sk, (const int8_t*)vt, (const _Float16*)sv,
                     (_Float16*)opart, (_Float16*)ml, (int)bh, (int)sq_tok, (int)sk_tok, group, ks, qks,
                     nullptr, nullptr);
  if constexpr (C::LIT_K > 0 && QA_FWD_DEFER) {   // the split rows whose first tile must be redone
    if (skip_fixup()) return hipGetLastError() == hipSuccess ? 0 : 2;
    auto fixk = int8_attn_fwd_kernel<D, false, true, false, true>;
    { static LdsGrant granted_; if (!lds_grant((const void*)fixk, lds, granted_)) return 1; }
    hipLaunchKernelGGL(fixk, dim3((unsigned)(nq * bh), (unsigned)nsplit), dim3(64 * C::WAVES), lds, st,
                       (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,
                       (const int8_t*)vt, (const _Float16*)sv, (_Float16*)opart, (_Float16*)ml, (int)bh,
                       (int)sq_tok, (int)sk_tok, group, ks, qks, nullptr, nullptr);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// q16 != nullptr: quantise q in the attention kernel (QF), writing q_i8, sq and (qbf != nullptr)
// the bf16 image
static int fwd_dispatch(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                        const void* vt, const void* sv, void* out, void* lse, long bh, long sq_tok,
                        long sk_tok, int group, int causal, int head_dim, float qks, const void* q16,
                        void* qbf, void* stream) {
  if (sq_tok % 32 != 0 || sk_tok % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128) || causal < 0 || causal > 2)
    return 1;
  if (bh == 0 || sq_tok == 0) return 0;
  if (sv == nullptr) return 1;
  if (sk_tok == 0 || (causal == 2 && sk_tok < sq_tok)) return 1;   // every query keeps a key
  const int qoff = causal == 2 ? (int)(sk_tok - sq_tok) : 0;
  hipStream_t st = (hipStream_t)stream;
  // Non-causal grouped-query attention with short query blocks: the group's query heads are
  // consecutive [sq_tok, D] blocks (rows, scale blocks, O and lse alike), so they run as one virtual
  // head of group * sq_tok rows against their key/value head -- the same arithmetic per row
  // (bit-identical), with the workgroup's waves filled and each key/value tile read once per group.
  if (causal == 0 && group > 1 && sq_tok % Int8FwdCfg<128>::QROWS != 0) {
    sq_tok *= group;
    bh /= group;
    group = 1;
  }
#define QA_L(Dv, CV, QV) \
  launch_fwd<Dv, CV, QV>(q_i8, sq, k_i8, sk, vt, sv, out, lse, bh, sq_tok, sk_tok, group, qoff, qks, \
                         q16, qbf, st)
  if (q16 != nullptr) {
    if (head_dim == 128) return causal ? QA_L(128, true, true) : QA_L(128, false, true);
    return causal ? QA_L(64, true, true) : QA_L(64, false, true);
  }
  if (head_dim == 128) return causal ? QA_L(128, true, false) : QA_L(128, false, false);
  return causal ? QA_L(64, true, false) : QA_L(64, false, false);
#undef QA_L
}

}  // namespace qattn

using namespace qattn;

#if QA_FWD_LIT_COUNT
extern "C" int qattn_fwd_lit_count(void* host_dst) {
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(qattn::g_fwd_lit), sizeof(qattn::g_fwd_lit)) == hipSuccess ? 0 : 2;
}
#endif
#if QA_FWD_STAMP
extern "C" int qattn_fwd_stamps(void* host_dst) {
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(qattn::g_fwd_stamp), sizeof(qattn::g_fwd_stamp)) == hipSuccess ? 0 : 2;
}
#endif

extern "C" int qattn_int8_attn_fwd_ex(const void* q_i8, const void* sq, const void* k_i8,
                                      const void* sk, const void* vt, const void* sv, void* out,
                                      void* lse, long bh, long sq_tok, long sk_tok, int group,
                                      int causal, int head_dim, float qks, void* stream) {
  return fwd_dispatch(q_i8, sq, k_i8, sk, vt, sv, out, lse, bh, sq_tok, sk_tok, group, causal,
                      head_dim, qks, nullptr, nullptr, stream);
}

extern "C" int qattn_int8_attn_fwd_qf(const void* q, void* q_i8, void* sq, void* q_bf, const void* k_i8,
                                      const void* sk, const void* vt, const void* sv, void* out,
                                      void* lse, long bh, long sq_tok, long sk_tok, int group,
                                      int causal, int head_dim, float qks, void* stream) {
  if ((q == nullptr || q_i8 == nullptr || sq == nullptr) && bh != 0 && sq_tok != 0) return 1;
  return fwd_dispatch(q_i8, sq, k_i8, sk, vt, sv, out, lse, bh, sq_tok, sk_tok, group, causal,
                      head_dim, qks, q, q_bf, stream);
}

extern "C" int qattn_int8_attn_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                                   const void* vt, const void* sv, void* out, void* lse, long bh,
                                   long seq, int head_dim, float qks, void* stream) {
  return qattn_int8_attn_fwd_ex(q_i8, sq, k_i8, sk, vt, sv, out, lse, bh, seq, seq, 1, 0, head_dim,
                                qks, stream);
}

// Key-split (flash-decoding) form of qattn_int8_attn_fwd_ex for short query blocks against long
// key ranges (the int8 key/value cache), non-causal: every workgroup covers
// keys_per_split keys (a multiple of 32) of its query rows and writes the partial state
//   opart f16 [nsplit][bh*sq_tok][D] = O_s / l_s and ml f32x2 [nsplit][bh*sq_tok] = {m_s, l_s},
// nsplit = ceil(sk_tok / keys_per_split); qattn_int8_split_combine merges it into out / lse.
// head_dim 128 only (the D = 64 instantiation exceeds the SGPR budget of its buffer descriptors).
extern "C" int qattn_int8_attn_fwd_split(const void* q_i8, const void* sq, const void* k_i8,
                                         const void* sk, const void* vt, const void* sv, void* opart,
                                         void* ml, long bh, long sq_tok, long sk_tok, int group,
                                         int keys_per_split, int head_dim, float qks, void* stream) {
  if (sv == nullptr || opart == nullptr || ml == nullptr || sq_tok % 32 != 0 || sk_tok % 32 != 0 ||
      group < 1 || bh % group != 0 || keys_per_split < 32 || keys_per_split % 32 != 0 ||
      head_dim != 128)
    return 1;
  if (bh == 0 || sq_tok == 0) return 0;
  if (sk_tok == 0) return 1;
  return launch_fwd_split<128>(q_i8, sq, k_i8, sk, vt, sv, opart, ml, bh, sq_tok, sk_tok, group,
                               keys_per_split, qks, (hipStream_t)stream);
}

extern "C" int qattn_int8_split_combine(const void* opart, const void* ml, void* out, void* lse, long rows,
                                        int nsplit, int head_dim, void* stream) {
  if (nsplit < 1 || (head_dim != 64 && head_dim != 128) || rows < 0) return 1;
  if (rows == 0) return 0;
  const long threads = rows * (head_dim / 8);
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL(int8_split_combine_kernel<128>, grid, dim3(256), 0, st, (const _Float16*)opart,
                       (const float2*)ml, (_Float16*)out, (_Float16*)lse, rows, nsplit);
  else
    hipLaunchKernelGGL(int8_split_combine_kernel<64>, grid, dim3(256), 0, st, (const _Float16*)opart,
                       (const float2*)ml, (_Float16*)out, (_Float16*)lse, rows, nsplit);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
