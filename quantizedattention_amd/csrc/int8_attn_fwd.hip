// SageAttention-3 int8 attention forward for gfx950 (replaces the attention part of
// helion_atten_int8_hl_dot_fwd, attention_int8.py:170-257), per (batch, head).
//
// Work decomposition
//   * one workgroup = 4 waves = 128 query rows of one (b,h); wave w owns rows 32w..32w+31 = one
//     32-token q-quant block (one sq scale per wave).  PV_I8: 2 workgroups per CU (<= 256 VGPRs);
//     PV_F16: 3 (<= 168 VGPRs).
//   * keys stream in 32-key tiles (= one Bkv block) through a 4-slot LDS ring filled by buffer
//     LDS-DMA (no staging registers; the bank swizzle is applied to the per-lane source offset, the
//     LDS image is written lane-linearly).  One barrier per tile; the DMA of tile t+3 is issued
//     right after the barrier of tile t.
//   * per-tile scales of the head sit in LDS (loaded once); workgroups of one head share an XCD.
//
// Per 32-key tile and wave (swapped orientation: keys in registers, query on the lane pair l, l^32),
// software-pipelined by one tile so that each wave has MFMA work beside its softmax VALU:
//     QK(t+1)   S^T = K_i8 . Q_i8^T                   D/32 x v_mfma_i32_32x32x32_i8
//     SM2(t)    e = exp2(d), l, P operand             (VALU, beside the QK(t+1) MFMAs)
//     PV(t)     O^T += V^T . P^T                      (PV modes below)
//     SM1(t+1)  d = S - rowmax, deferred running max  (VALU, beside the PV(t) MFMAs)
// Reference rounding points (int8:197-257):
//     S  = f16(acc * c),  c = sq*sk*qks          on the biased accumulator: one v_pk_fma_f32 per pair
//                                                + v_cvt_pk_f16_f32 (QA_FWD_S_PK, default), or one
//                                                v_fma_mix per score
//                                                (common.h KMAG: no int -> float conversion)
//     rm = f16(max_k(acc) * c)                   (c > 0: the row max commutes with the scaling)
//     d  = f16(S - rm)                           (S rounded to f16 first, as the reference does)
//     e  = exp2(d);  P_i8 = trunc(127 e);  sp = exp2(rm - m)/127  (int8:211-237)
//     l += exp2(rm - m) * sum e (fp32);  O *= exp2(m_old - m) when the running max moves.
// Deferred max (cdna_hip_programming.md T13): the running max m moves only when some row's tile max
// exceeds it by more than THR = 8 (log2 units); P_i8 depends only on S - rowmax(tile), O and l share
// the (possibly stale) reference, so O / l is unchanged up to rounding.
//
// P.V modes (int8:249-250, O += (P_i8 . v_i8) * sp * sv per 32-key tile):
//   PV_F16            one v_mfma_f32_32x32x16_f16 chain on f16(P_i8 * sp) x f16(v_i8 * sv) (the
//                     quantiser's vdq image): the tile scale rides in the operands, the fp32
//                     accumulator needs no per-tile work.  P_i8 and the scales are the reference's;
//                     the extra rounding is that of the two f16 products.
//   PV_I8 (default)   the literal reference contraction: v_mfma_i32_32x32x32_i8 on P_i8 x v_i8 (V^T
//                     operand image vt from qattn_int8_quant_vt), exact int32 per tile, then one
//                     fused dequantisation per accumulator element and tile, O += acc * sp*sv
//                     (biased accumulator: 1 VALU per element instead of 2).
//   Both keep the reference's per-32-key P quantisation; coarser P.V blocks (one dequantisation per
//   2 or 4 tiles) move O by 1.3e-2 .. 6e-2 from the reference (tools/pv_quant_study.py: the
//   truncation bias grows with the block), past the 1e-2 bar.  PV_I8 spends 32 packed fp32 FMAs per
//   wave-tile on the dequantisation but streams half the V bytes (int8 image, 4 KiB per tile through
//   DMA and LDS instead of 8) and issues 8 MFMAs instead of 12: measured 15-18 % faster than PV_F16
//   at config 3.
#include <climits>
#include <type_traits>

#include "common.h"
#include "int8_fwd_plan.h"

namespace qattn {

// (compiles to v_max3_i32).  Deliberately NOT inline asm: its inputs are MFMA results, and hipcc's
// hazard recogniser inserts the MFMA-result -> VALU wait states only for instructions it emits itself.
QA_DEVICE int imax3(int a, int b, int c) { return max(max(a, b), c); }

// Per-wave softmax state between the two halves of a tile.
struct SmTile {
  v2h d[8];       // f16(S - rm) for the 16 scores of this lane
  float er;       // exp2(rm - m)
  float cpv;      // PV_F16: sp = f16(er / 127) (as f32); PV_I8: the tile's dequantisation er/127*sv
  v2h pi[8];      // CAUSAL diagonal tiles: P_i8 by the reference's literal chain (f16 integers)
  bool diag;      // (wave-uniform) this tile crosses the wave's causal diagonal
};

// Shapes: BH = batch * query heads, Sq query and Sk key tokens per head; query head
// bh reads key/value head bh / G (grouped-query attention, G = Hq / Hkv).  CAUSAL keeps key <=
// query + qoff: qoff = 0 aligns the first query with the first key (top-left), qoff = Sk - Sq the
// last with the last (bottom-right: new queries against a key/value cache); masked
// scores are excluded (P = 0).  The reference has neither (its int8 path is square, ungrouped and
// non-causal, int8:122-127, 344); these are extensions.
// vop: PV_F16 the vdq image f16 [BHkv*Sk, D]; PV_I8 the vt image (qattn_int8_quant_vt).
// SPLIT (key-split decoding, PV_I8 non-causal): workgroup (x, y) covers keys [y ks, y ks + ks) of
// its query rows and writes the partial state instead of O: through `out`, opart f16
// [split][BH*Sq][D] = f16(O_s / l_s) (the split's normalised output); through `lse`, ml f32x2
// [split][BH*Sq] = {m_s, l_s} (running max, row sum); int8_split_combine_kernel merges the splits.  (The two
// outputs reuse the pointer arguments and ks the causal offset qoff: the causal instantiations are
// at the SGPR limit, one more kernel argument pushes their buffer descriptors into VGPRs.)
// (the causal PV_F16 kernel's diagonal masking does not fit 168 VGPRs: 2 waves per SIMD)
template <int D, int PV, bool CAUSAL>
constexpr int fwd_wps() { return CAUSAL ? 2 : Int8FwdCfg<D, PV>::WPS; }
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
template <int D, int PV, bool CAUSAL, bool SPLIT = false>
__global__ __launch_bounds__((64 * Int8FwdCfg<D, PV>::WAVES), (fwd_wps<D, PV, CAUSAL>())) void int8_attn_fwd_kernel(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const void* __restrict__ vop, const _Float16* __restrict__ sv,
    _Float16* __restrict__ out, _Float16* __restrict__ lse, int BH, int Sq, int Sk, int G, int qoff,
    float qks) {
  static_assert(!SPLIT || (PV == PV_I8 && !CAUSAL), "key splits: int8 P.V, non-causal");
  using C = Int8FwdCfg<D, PV>;
  FWD_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // per-tile scales: ck = sk * qks (f32); PV_I8 also sv / 127 (f32)
  float* ck_lds = reinterpret_cast<float*>(smem + C::RING);

  const int nq = (Sq + C::QROWS - 1) / C::QROWS;
  int bh, qt;
  if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nq, BH, true, bh, qt);
  else xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int q0 = qt * C::QROWS + wave * 32;
  const bool active = q0 < Sq;
  const long head_row0 = (long)bh * Sq;           // this head's query rows
  const int split = SPLIT ? (int)__builtin_amdgcn_readfirstlane(blockIdx.y) : 0;
  const int ks = qoff;                             // SPLIT (non-causal): keys per split
  const int k0 = SPLIT ? split * ks : 0;           // first key of this workgroup's key range
  const int nk = SPLIT ? min(ks, Sk - k0) : Sk;    // its keys
  const long kv_row0 = (long)(bh / G) * Sk + k0;  // its key/value head's rows
  const int8_t* kbase = k_i8 + kv_row0 * D;
  const void* vbase = PV == PV_F16
      ? (const void*)(reinterpret_cast<const _Float16*>(vop) + kv_row0 * D)
      : (const void*)(reinterpret_cast<const int8_t*>(vop) + kv_row0 * D);
  // causal: key tiles past the workgroup's last query are masked for all of its rows
  const int nt = CAUSAL ? min(Sk / C::KT, (qt * C::QROWS + C::QROWS + qoff + C::KT - 1) / C::KT)
                        : nk / C::KT;
  // per-tile scales, shifted by one tile: entry i holds tile min(i + 1, nt - 1), the tile whose SM1
  // runs in loop iteration i, so that 4 iterations read their scales with one 16-B LDS read
  float* svq_lds = ck_lds + ((nt + 3) & ~3);

  DmaPlan<D, PV> dma;
  dma.init(wave, lane, Sk - k0, kbase, vbase);   // (the range bound only: reads stay in nk)
  const unsigned smem_lds = lds_addr(smem);
  dma.issue(smem_lds, 0);
  dma.issue(smem_lds + 1 * C::SLOT, min(1, nt - 1));
  dma.issue(smem_lds + 2 * C::SLOT, min(2, nt - 1));
  for (int i = tid; i < nt; i += 64 * C::WAVES) {
    const int ti = min(i + 1, nt - 1);
    ck_lds[i] = (float)sk[kv_row0 / 32 + ti] * qks;
    if constexpr (PV == PV_I8) svq_lds[i] = (float)sv[kv_row0 / 32 + ti] * (1.0f / 127.0f);
  }
  const float ck0 = (float)sk[kv_row0 / 32] * qks;   // tile 0 (the prologue's SM1)
  const float svq0 = PV == PV_I8 ? (float)sv[kv_row0 / 32] * (1.0f / 127.0f) : 0.f;

  // ---- Q fragment (B operand of S^T = K Q^T): lane holds Q[q0+c32][32s + 16h .. +16]
  v4i qf[C::NKS];
  float cq = 0.f;
  if (active) {
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

  // lane-constant LDS byte offsets: K A-operand chunk (2s+h) of key row c32; PV_F16: V^T A-operand
  // of d-block b: key rows 4h + (i16>>2) (+16 per k-step, +8 for the 2nd read), columns
  // 32b + 16gg + 4(i16&3); PV_I8: piece b of the vt image, 16 B per lane
  int koff[C::NKS], voff[C::NDB];
#pragma unroll
  for (int s = 0; s < C::NKS; ++s) koff[s] = c32 * D + 16 * ((2 * s + h) ^ k_sw<D>(c32));
  if constexpr (PV == PV_F16) {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int key_a = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      voff[b] = C::K_BYTES + key_a * 2 * D + 16 * ((d / 8) ^ v_sw<D>(key_a)) + (d % 8) * 2;
    }
  } else {
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) voff[b] = C::K_BYTES + b * 1024 + 16 * lane;
  }

  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  _Float16 m = (_Float16)(-INFINITY);
  _Float16 m_thr = (_Float16)(-INFINITY);   // m + THR (f16): the deferred running max moves past it
  _Float16 mt = (_Float16)(-INFINITY);   // CAUSAL: the reference's (undeferred) running max
  float l = 0.f;      // per-lane partial (this lane's key half); the reference's l = 1 is wiped by r = 0
  float obias = 0.f;  // PV_I8: sum of the tile dequantisation factors (the KMAG bias of O is KMAG * obias)
  // PV_I8: the dequantisation factor of the tile whose P.V is in flight while SM1 of the next tile
  // runs; a running-max move there rescales it with O (its int32 product is added after SM1)
  float cpv_pend = 0.f;

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
    v16i acc = mfma_i8(kf[0], qf[0], C::QK_BIAS ? kmag : v16i{});
#pragma unroll
    for (int s = 1; s < C::NKS; ++s) acc = mfma_i8(kf[s], qf[s], acc);
    return acc;
  };

  // first half of the softmax of tile t: row max, d = f16(S - rm), deferred running max, er, and
  // the tile's P.V scale
  //   dg (std::true_type / false_type): whether tile t may cross the diagonal (causal), i.e.
  //   whether the masks and the literal P chain are compiled in
  auto sm1 = [&](const v16i& acc_in, int t, SmTile& st, float ckt, float svqt, auto dg) {
    // causal tiles crossing this wave's diagonal: keys above the row's query drop out of the max
    // (INT_MIN) and get d = -inf below, so P = 0 and the tile scale ignores them
    const bool diag = CAUSAL && decltype(dg)::value && (t * C::KT + C::KT - 1 > q0 + qoff);
    // QA_FWD_LITERAL_P: the reference's literal P_i8 chain on every tile (priced)
    const bool lit = diag || (QA_FWD_LITERAL_P != 0);
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
    // S = f16(X * c) (int8:200-203: fp32 products, then fp16)
    v2h s2[8];
    _Float16 rm;
    if constexpr (C::QK_BIAS) {   // on the biased accumulator (QA_FWD_S_PK: packed f32, else fma_mix)
      const float c = kmag_scale(cq * ckt);
      const float nb = -KMAG * c;
#if QA_FWD_S_PK
      rm = biased_to_f16(mx, c, nb);
      biased_to_f16x16(acc, c, nb, s2);
#else
      rm = fma_mix1(__int_as_float(mx), c, nb);
      fma_mix16_after(acc, c, nb, mx, s2);
#endif
    } else {
      const float c = cq * ckt;
      rm = (_Float16)((float)mx * c);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        s2[j] = __builtin_bit_cast(v2h, pk_f16((float)acc[2 * j] * c, (float)acc[2 * j + 1] * c));
    }
    const v2h rm2 = {rm, rm};
#pragma unroll
    for (int j = 0; j < 8; ++j) st.d[j] = s2[j] - rm2;   // f16(S - rm)  (int8:211, 232-236)
    if constexpr (CAUSAL || QA_FWD_LITERAL_P) {
      // Diagonal tiles keep few keys per row, where one P_i8 step weighs much in O: there P_i8
      // follows the reference chain literally (int8:205-237): next_m = max(m, rm) with the
      // undeferred running max, P = exp2(f32(f16(S - next_m))), sp = exp2(f32(f16(rm - next_m)))/127
      // and P_i8 = trunc(P / sp), IEEE fp32 divisions.  Other tiles use 127 exp2(f16(S - rm)) (the
      // same value up to the last bits, which only matter when few keys share the row sum).
      const bool kept = mx != INT_MIN;     // the row keeps a key of this tile
      const _Float16 nm_ref = (kept && rm > mt) ? rm : mt;
      if (kept) mt = nm_ref;
      st.diag = lit;
      if (lit) {
        const float spr = exp2_f32((float)(_Float16)((float)rm - (float)nm_ref)) / 127.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float dr = (float)(_Float16)((float)s2[j][e] - (float)nm_ref);
            const float pr = __builtin_truncf(exp2_f32(dr) / spr);
            st.pi[j][e] = (acc[2 * j + e] == INT_MIN || !kept) ? (_Float16)0.0f : (_Float16)pr;
          }
      }
    }
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
      if constexpr (PV == PV_I8) {
        obias *= r;
        cpv_pend *= r;
      }
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) o[b] *= r;
    }
    st.er = exp2_f32((float)(_Float16)(rm - m));
    if constexpr (PV != PV_I8) st.cpv = (float)(_Float16)(st.er * (1.0f / 127.0f));
    else st.cpv = st.er * svqt;
  };

  // second half: e = exp2(d) (sm2_exp), then l += er * sum e and the P operand (sm2)
  //   PV_F16: f16(P_i8 * sp) as 2 x 4 packed dwords; PV_I8: the 16 P_i8 bytes
  auto sm2_exp = [&](const SmTile& st, v2h* e) {
    exp2_pk4(&st.d[0], &e[0]);
    exp2_pk4(&st.d[4], &e[4]);
  };
  auto sm2 = [&](const SmTile& st, const v2h* e, v4u* pw) {
    // row sum of e: packed f16 adds (pairs, then sums of 4 and 8 values <= 8), one f32 mix-add
    const v2h s = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
    l = fmaf(pk_hsum(s), st.er, l);
    if ((CAUSAL || QA_FWD_LITERAL_P) && st.diag) {   // the literal-chain P_i8 of the tile (sm1)
      if constexpr (PV != PV_I8) {
        const _Float16 sp = (_Float16)st.cpv;
        const v2h sp2 = {sp, sp};
#pragma unroll
        for (int j = 0; j < 8; ++j) pw[j / 4][j % 4] = __builtin_bit_cast(unsigned, st.pi[j] * sp2);
      } else {
        const v2h k1024 = {(_Float16)1024.0f, (_Float16)1024.0f};
        unsigned y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = __builtin_bit_cast(unsigned, st.pi[j] + k1024);
        pw[0] = __builtin_bit_cast(v4u, pack_p_index(y));
      }
      return;
    }
    if constexpr (PV != PV_I8) {
      const _Float16 sp = (_Float16)st.cpv;
      const v2h sp2 = {sp, sp};
      const _Float16 nsp = (_Float16)(-1024.0f) * sp;
      const v2h nsp2 = {nsp, nsp};
      v2h w[8];
      p_operand8(e, sp2, nsp2, w);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) pw[u][j] = __builtin_bit_cast(unsigned, w[4 * u + j]);
    } else {
      const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
      unsigned y[8];
      p_index8(e, k127, y);
      pw[0] = __builtin_bit_cast(v4u, pack_p_index(y));
    }
  };

  // O^T += V^T P^T for tile t: operand loads (issued early, consumed after QK(t+1) and SM2(t))
  // and the MFMAs
  using VFrag = typename std::conditional<PV != PV_I8, v8h, v4i>::type;
  constexpr int NVF = PV != PV_I8 ? 2 * C::NDB : C::NDB;
  auto pv_load = [&](int u, VFrag* va) {
    const char* vl = slot_at(u);
    if constexpr (PV == PV_F16) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) {
          const char* a = vl + voff[b] + 16 * s * 2 * D;
          va[s * C::NDB + b] = __builtin_bit_cast(v8h, ds_read_tr16_x2(a, a + 8 * 2 * D));
        }
    } else {
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) va[b] = *reinterpret_cast<const v4i*>(vl + voff[b]);
    }
  };
  v16i pacc[PV == PV_I8 ? C::NDB : 1];
  auto pv_mma = [&](const VFrag* va, const v4u* pw) {
    if constexpr (PV != PV_I8) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int b = 0; b < C::NDB; ++b)
          o[b] = mfma_f16(va[s * C::NDB + b], __builtin_bit_cast(v8h, pw[s]), o[b]);
    } else {
      const v4i p = __builtin_bit_cast(v4i, pw[0]);
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) pacc[b] = mfma_i8(va[b], p, kmag);
    }
  };
  // PV_I8: O += (KMAG + X) * (sp * sv) for the tile's exact int32 X (one fused op per element)
  auto pv_dequant = [&](float cpv) {
    if constexpr (PV == PV_I8) {
      // explicit v_pk_fma_f32 pairs (scalar v_fma_f32 measured 2-3 % slower)
      const v2f_ c2 = {cpv, cpv};
#pragma unroll
      for (int b = 0; b < C::NDB; ++b)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          const v2f_ a = {__int_as_float(pacc[b][r]), __int_as_float(pacc[b][r + 1])};
          const v2f_ y = __builtin_elementwise_fma(a, c2, v2f_{o[b][r], o[b][r + 1]});
          o[b][r] = y[0];
          o[b][r + 1] = y[1];
        }
      obias += cpv;
    }
  };

  vmem_drain();
  __syncthreads();
  FWD_STAMP(1);

  SmTile st;
  // One loop iteration per tile t: SM2 and P.V of tile t, QK and SM1 of tile t+1.  The last iteration
  // computes QK / SM1 of a duplicate of the last tile (its slot holds a clamped re-load): harmless
  // (its row max cannot move m) and it keeps the loop body branch-free.
  //   cur, nxt: ring slots of tiles t and t+1; fill: the slot the DMA of tile t+3 goes to (freed by
  //   the barrier); ckn, svqn: the scales of tile t+1
  auto iter = [&](int t, int cur, int nxt, int fill, float ckn, float svqn, auto dg) {
    ring_wait_barrier<C::IPW>();   // tile t+1 landed (t+2 may be in flight); slot `fill` is free
    dma.issue(smem_lds + fill * C::SLOT, min(t + 3, nt - 1));
    // Phase order (pinned: hipcc otherwise issues the QK(t+1) chain right before its consumer
    // SM1(t+1) and the wave stalls on it): fragment reads, the 16 exponentials of tile t (which
    // cover the LDS latency), QK(t+1), then the rest of SM2(t), PV(t) and SM1(t+1).
    const int tn = min(t + 1, nt - 1);
    v4i kf[C::NKS];
    qk_load(nxt, kf);
    VFrag va[NVF];
    pv_load(cur, va);
    v2h e[8];
    sm2_exp(st, e);
    __builtin_amdgcn_sched_barrier(0);
    const v16i nacc = qk_mma(kf);
    __builtin_amdgcn_sched_barrier(0);
    v4u pw[2];
    sm2(st, e, pw);
    cpv_pend = st.cpv;
    pv_mma(va, pw);
    sm1(nacc, tn, st, ckn, svqn, dg);   // (may rescale O, obias and cpv_pend)
    pv_dequant(cpv_pend);   // PV_I8: after SM1(t+1), so the PV MFMAs of tile t have retired
  };
  if (active) {
    {
      v4i kf[C::NKS];
      qk_load(0, kf);
      sm1(qk_mma(kf), 0, st, ck0, svq0, std::true_type{});
    }
    // Causal: iteration t runs SM1 of tile t+1, and tiles below td0 = (first query of the workgroup
    // + qoff) / KT cross no wave's diagonal, so iterations t < td0 - 1 run with the masks and the
    // literal P chain compiled out (the same values: nothing is masked there) and the rest, at
    // most WAVES + 1 of them, with them.
    const int tmain = CAUSAL ? max(0, min(nt, (qt * C::QROWS + qoff) / C::KT - 1)) : nt;
    // groups of NSLOT = 4 tiles with compile-time ring slots (immediate LDS offsets, one 16-B read
    // of each scale table per group), then the remaining tiles with run-time slots.  Only where the
    // unrolled body fits the register budget (the 3-wave f16 P.V kernel spills with it).
    static_assert(C::NSLOT == 4, "ring of 4 slots");
    constexpr bool UNROLL = PV == PV_I8 && QA_FWD_UNROLL;
    const std::false_type nodiag{};
    int t = 0;
    for (; UNROLL && t + 4 <= tmain; t += 4) {
      const v4f ck4 = *reinterpret_cast<const v4f*>(ck_lds + t);
      const v4f sv4 = PV == PV_I8 ? *reinterpret_cast<const v4f*>(svq_lds + t) : v4f{};
      iter(t, 0, 1, 3, ck4[0], sv4[0], nodiag);
      iter(t + 1, 1, 2, 0, ck4[1], sv4[1], nodiag);
      iter(t + 2, 2, 3, 1, ck4[2], sv4[2], nodiag);
      iter(t + 3, 3, 0, 2, ck4[3], sv4[3], nodiag);
    }
    for (; t < tmain; ++t)
      iter(t, t & 3, (t + 1) & 3, (t + 3) & 3, ck_lds[t], PV == PV_I8 ? svq_lds[t] : 0.f, nodiag);
    if constexpr (CAUSAL) {
      for (; t < nt; ++t)
        iter(t, t & 3, (t + 1) & 3, (t + 3) & 3, ck_lds[t], PV == PV_I8 ? svq_lds[t] : 0.f,
             std::true_type{});
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
  if constexpr (SPLIT) {   // the partial state of this key range: {m, l} and f16(O / l)
    l = pair_sum(l);
    const long prow = ((long)split * BH + bh) * Sq + q0;
    if (h == 0) reinterpret_cast<float2*>(lse)[prow + c32] = float2{(float)m, l};
    const float inv = 1.0f / l;
    store_rows<D, _Float16, 1, true>(o, inv, smem + wave * RowTile<D, _Float16>::BYTES,
                                     out + prow * D, lane, -KMAG * obias * inv);
    return;
  }
  // ---------------- epilogue: lse = fp16(m + fp16(log2 l)); O = fp16(O / l)   (int8:252-257)
  l = pair_sum(l);
  const long qrow = head_row0 + q0 + c32;
  if (h == 0) lse[qrow] = (_Float16)((float)m + (float)(_Float16)log2_f32(l));
  const float inv = 1.0f / l;
  store_rows<D, _Float16, 1, PV == PV_I8>(o, inv, smem + wave * RowTile<D, _Float16>::BYTES,
                                          out + (head_row0 + q0) * D, lane, -KMAG * obias * inv);
#if QA_FWD_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  FWD_STAMP(3);
#endif
}

template <int D, int PV, bool CAUSAL>
static int launch_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                      const void* vop, const void* sv, void* out, void* lse, long bh, long sq_tok,
                      long sk_tok, int group, int qoff, float qks, hipStream_t st) {
  using C = Int8FwdCfg<D, PV>;
  const int nq = (int)((sq_tok + C::QROWS - 1) / C::QROWS);
  const int lds = C::RING + (int)((((sk_tok / 32) + 3) / 4 * 4) * 4 * (PV == PV_I8 ? 2 : 1));
  { static int granted_ = 0; lds_grant((const void*)int8_attn_fwd_kernel<D, PV, CAUSAL>, lds, granted_); }
  hipLaunchKernelGGL((int8_attn_fwd_kernel<D, PV, CAUSAL>), dim3((unsigned)(nq * bh)),
                     dim3(64 * C::WAVES), lds, st, (const int8_t*)q_i8, (const _Float16*)sq,
                     (const int8_t*)k_i8, (const _Float16*)sk, vop, (const _Float16*)sv,
                     (_Float16*)out, (_Float16*)lse, (int)bh, (int)sq_tok, (int)sk_tok, group, qoff, qks);
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
  using C = Int8FwdCfg<D, PV_I8>;
  const int nq = (int)((sq_tok + C::QROWS - 1) / C::QROWS);
  const int nsplit = (int)((sk_tok + ks - 1) / ks);
  const int lds = C::RING + (int)((((ks / 32) + 3) / 4 * 4) * 8);
  { static int granted_ = 0; lds_grant((const void*)int8_attn_fwd_kernel<D, PV_I8, false, true>, lds, granted_); }
  hipLaunchKernelGGL((int8_attn_fwd_kernel<D, PV_I8, false, true>), dim3((unsigned)(nq * bh), (unsigned)nsplit),
                     dim3(64 * C::WAVES), lds, st, (const int8_t*)q_i8, (const _Float16*)sq,
                     (const int8_t*)k_i8, (const _Float16*)sk, vt, (const _Float16*)sv, (_Float16*)opart,
                     (_Float16*)ml, (int)bh, (int)sq_tok, (int)sk_tok, group, ks, qks);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

template <int PV>
static int fwd_dispatch(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                        const void* vop, const void* sv, void* out, void* lse, long bh, long sq_tok,
                        long sk_tok, int group, int causal, int head_dim, float qks, void* stream) {
  if (sq_tok % 32 != 0 || sk_tok % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128) || causal < 0 || causal > 2)
    return 1;
  if (bh == 0 || sq_tok == 0) return 0;
  if (sk_tok == 0 || (causal == 2 && sk_tok < sq_tok)) return 1;   // every query keeps a key
  const int qoff = causal == 2 ? (int)(sk_tok - sq_tok) : 0;
  hipStream_t st = (hipStream_t)stream;
  // Non-causal grouped-query attention with short query blocks: the group's query heads are
  // consecutive [sq_tok, D] blocks (rows, scale blocks, O and lse alike), so they run as one virtual
  // head of group * sq_tok rows against their key/value head -- the same arithmetic per row
  // (bit-identical), with the workgroup's waves filled and each key/value tile read once per group.
  if (causal == 0 && group > 1 && sq_tok % Int8FwdCfg<128, PV>::QROWS != 0) {
    sq_tok *= group;
    bh /= group;
    group = 1;
  }
#define QA_L(Dv, CV) \
  launch_fwd<Dv, PV, CV>(q_i8, sq, k_i8, sk, vop, sv, out, lse, bh, sq_tok, sk_tok, group, qoff, qks, st)
  if (head_dim == 128) return causal ? QA_L(128, true) : QA_L(128, false);
  return causal ? QA_L(64, true) : QA_L(64, false);
#undef QA_L
}

}  // namespace qattn

using namespace qattn;

#if QA_FWD_STAMP
extern "C" int qattn_fwd_stamps(void* host_dst) {
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(qattn::g_fwd_stamp), sizeof(qattn::g_fwd_stamp)) == hipSuccess ? 0 : 2;
}
#endif

extern "C" int qattn_int8_attn_fwd_ex(const void* q_i8, const void* sq, const void* k_i8,
                                      const void* sk, const void* vdq, void* out, void* lse, long bh,
                                      long sq_tok, long sk_tok, int group, int causal, int head_dim,
                                      float qks, void* stream) {
  return fwd_dispatch<PV_F16>(q_i8, sq, k_i8, sk, vdq, nullptr, out, lse, bh, sq_tok, sk_tok, group,
                              causal, head_dim, qks, stream);
}

extern "C" int qattn_int8_attn_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                                   const void* vdq, void* out, void* lse, long bh, long seq,
                                   int head_dim, float qks, void* stream) {
  return qattn_int8_attn_fwd_ex(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, 0, head_dim, qks,
                                stream);
}

extern "C" int qattn_int8_attn_fwd_i8pv_ex(const void* q_i8, const void* sq, const void* k_i8,
                                           const void* sk, const void* vt, const void* sv, void* out,
                                           void* lse, long bh, long sq_tok, long sk_tok, int group,
                                           int causal, int head_dim, float qks, void* stream) {
  if (sv == nullptr && bh > 0 && sq_tok > 0) return 1;   // (empty problems: nothing to read)
  return fwd_dispatch<PV_I8>(q_i8, sq, k_i8, sk, vt, sv, out, lse, bh, sq_tok, sk_tok, group, causal,
                             head_dim, qks, stream);
}

// Key-split (flash-decoding) form of qattn_int8_attn_fwd_i8pv_ex for short query blocks against
// long key ranges (the int8 key/value cache), non-causal: every workgroup covers
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
