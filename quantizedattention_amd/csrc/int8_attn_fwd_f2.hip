// SageAttention-3 int8 attention forward for gfx950, P.V on the f16 MFMA, software-pipelined by
// TWO key tiles (replaces the attention part of helion_atten_int8_hl_dot_fwd, attention_int8.py:
// 170-257; non-causal).  Same arithmetic as the PV_F16 mode of int8_attn_fwd.hip with the biased S
// accumulator (QA_FWD_QK_BIAS=1): bit-identical O and lse (tests/test_gpu_int8.py).
//
// Why a second schedule.  In int8_attn_fwd.hip every wave runs, per 32-key tile t,
//     QK(t+1) -> SM2(t) -> PV(t) -> SM1(t+1)
// and SM1(t+1) consumes the QK(t+1) MFMAs issued a few instructions earlier, so each wave spends a
// phase blocked behind its own matrix work; with one barrier per tile both waves of a SIMD reach that
// phase together and the SIMD idles (PMC: 50 % of wave-cycles in SQ_WAIT_INST_ANY for the f16 mode).
// Here the softmax of tile t reads S(t), produced one step EARLIER:
//     step t:   MFMA   QK(t+1) -> S(t+1)         (4 x v_mfma_i32_32x32x32_i8, K(t+1) from LDS)
//                      PV(t-1) with P(t-1)       (2 D/32 x v_mfma_f32_32x32x16_f16, V(t-1) from LDS)
//               VALU   softmax of S(t) -> P(t)   (no operand of this step's MFMAs)
// so the 12 MFMAs and the ~95 vector instructions of a step are independent and are issued
// interleaved, one MFMA per group of vector instructions (sched_barrier-pinned groups below): the
// matrix pipe runs while the wave issues its softmax.  Cost: a second S accumulator and P operand
// (unrolled by two, no register copies) and a 5-slot LDS ring (tiles t-1 .. t+3 live).
//
// The running max stays deferred (THR, int8_fwd_plan.h).  The P operand of tile t needs
// er = exp2(rm - m); it is computed with the current m before the (rare) rescale branch, and the
// branch -- which comes after this step's P.V MFMAs in program order, so O holds P(t-1).V(t-1) at
// the old reference when it is rescaled -- recomputes l and P(t) from the saved pieces.
#include <climits>

#include "common.h"
#include "int8_fwd_plan.h"

namespace qattn {

template <int D>
struct F2Cfg {
  using B = Int8FwdCfg<D, PV_F16>;
  static_assert(B::WAVES == 4, "4-wave workgroups (DmaPlan)");
  static constexpr int NSLOT = 5;
  static constexpr int STAGE = 4 * RowTile<D, _Float16>::BYTES;
  static constexpr int RING = NSLOT * B::SLOT > STAGE ? NSLOT * B::SLOT : STAGE;
};

// f16(a * c + n) of the even / odd scores of a biased accumulator into the low / high halves of
// r[j] (v_fma_mix{lo,hi}_f16, one rounding: as fma_mix16_after, split so that an MFMA can sit
// between the halves).  `dep` orders the asm after a compiler-emitted read of the accumulator (hipcc
// inserts MFMA-result -> VALU wait states only for its own instructions).
QA_DEVICE void mix8_lo(const v16i& acc, float c, float n, int dep, unsigned* r) {
  asm("v_fma_mixlo_f16 %0, %8, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %1, %9, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %2, %10, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %3, %11, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %4, %12, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %5, %13, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %6, %14, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixlo_f16 %7, %15, %16, %17 op_sel_hi:[0,0,0]"
      : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]),
        "=&v"(r[7])
      : "v"(acc[0]), "v"(acc[2]), "v"(acc[4]), "v"(acc[6]), "v"(acc[8]), "v"(acc[10]),
        "v"(acc[12]), "v"(acc[14]), "v"(c), "v"(n), "v"(dep));
}
QA_DEVICE void mix8_hi(const v16i& acc, float c, float n, unsigned* r) {
  asm("v_fma_mixhi_f16 %0, %8, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %1, %9, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %2, %10, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %3, %11, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %4, %12, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %5, %13, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %6, %14, %16, %17 op_sel_hi:[0,0,0]\n\t"
      "v_fma_mixhi_f16 %7, %15, %16, %17 op_sel_hi:[0,0,0]"
      : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]),
        "+v"(r[7])
      : "v"(acc[1]), "v"(acc[3]), "v"(acc[5]), "v"(acc[7]), "v"(acc[9]), "v"(acc[11]),
        "v"(acc[13]), "v"(acc[15]), "v"(c), "v"(n));
}

#define QA_F2_FENCE() __builtin_amdgcn_sched_barrier(0)
// S = f16(X c) through v_pk_fma_f32 + v_cvt_pk_f16_f32 (1) or v_fma_mix{lo,hi}_f16 (0)
#ifndef QA_F2_S_PK
#define QA_F2_S_PK 1
#endif
// Timing-only ablations (tools/ab_build.sh; wrong results): 1 no workgroup barrier per step, 2 no V
// LDS reads, 4 no K LDS reads, 8 no DMA
#ifndef QA_F2_ABL
#define QA_F2_ABL 0
#endif

template <int D>
__global__ __launch_bounds__(256, 2) void int8_attn_fwd_f2_kernel(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const _Float16* __restrict__ vdq, _Float16* __restrict__ out,
    _Float16* __restrict__ lse, int BH, int Sq, int Sk, int G, float qks) {
  using C = Int8FwdCfg<D, PV_F16>;
  using F = F2Cfg<D>;
  constexpr int NS = F::NSLOT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* ck_lds = reinterpret_cast<float*>(smem + F::RING);   // ck = sk * qks per key tile

  const int nq = (Sq + C::QROWS - 1) / C::QROWS;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int q0 = qt * C::QROWS + wave * 32;
  const bool active = q0 < Sq;
  const long head_row0 = (long)bh * Sq;
  const long kv_row0 = (long)(bh / G) * Sk;
  const int nt = Sk / C::KT;

  DmaPlan<D, PV_F16> dma;
  dma.init(wave, lane, Sk, k_i8 + kv_row0 * D, vdq + kv_row0 * D);
  const unsigned smem_lds = lds_addr(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i) dma.issue(smem_lds + i * C::SLOT, min(i, nt - 1));
  for (int i = tid; i < nt; i += 256) ck_lds[i] = (float)sk[kv_row0 / 32 + i] * qks;

  // Q fragment (B operand of S^T = K Q^T): lane holds Q[q0+c32][32s + 16h .. +16]
  v4i qf[C::NKS];
  float cq = 0.f;
  if (active) {
    const int8_t* qrow = q_i8 + (head_row0 + q0 + c32) * D + 16 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v4i*>(qrow + 32 * s);
    cq = (float)sq[(head_row0 + q0) / 32];
  }
  v16i kmag;
#pragma unroll
  for (int i = 0; i < 16; ++i) kmag[i] = KMAG_BITS;
  asm volatile("" : "+v"(kmag));

  // lane-constant LDS offsets (as int8_attn_fwd.hip PV_F16): K A-operand chunk (2s+h) of key row
  // c32; V^T A-operand of d-block b (key rows 4h + (i16>>2), +16 per k-step, +8 for the 2nd read)
  int koff[C::NKS], voff[C::NDB];
#pragma unroll
  for (int s = 0; s < C::NKS; ++s) koff[s] = c32 * D + 16 * ((2 * s + h) ^ k_sw<D>(c32));
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int key_a = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      voff[b] = C::K_BYTES + key_a * 2 * D + 16 * ((d / 8) ^ v_sw<D>(key_a)) + (d % 8) * 2;
    }
  }

  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  _Float16 m = (_Float16)(-INFINITY);
  float l = 0.f;
  float ck_cur = 0.f;   // ck of the tile whose softmax runs next (read one step ahead)
  float mthr = -INFINITY;   // (float)m + THR: the running max moves when a row's tile max passes it

  // LDS reads of a ring slot: one address add per lane-constant offset, made opaque so that hipcc
  // keeps the per-read constants as ds immediates (instead of hoisting one address VGPR per read)
  typedef __attribute__((address_space(3))) const char lds_byte;
  const unsigned sbase = smem_lds;
  auto slot_off = [&](int t) { return (int)__builtin_amdgcn_readfirstlane((t % NS) * C::SLOT); };
  auto qk_load = [&](int so, v4i* kf) {
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
      unsigned a = sbase + koff[s] + so;
      asm("" : "+v"(a));
      kf[s] = *(__attribute__((address_space(3))) const v4i*)(uintptr_t)a;
    }
  };
  auto pv_load = [&](int so, v8h* va) {
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      unsigned a = sbase + voff[b] + so;
      asm("" : "+v"(a));
      lds_byte* p = (lds_byte*)(uintptr_t)a;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        typedef __attribute__((address_space(3))) v4s lds_v4s;
        const v4s r0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p + 16 * s * 2 * D));
        const v4s r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p + 16 * s * 2 * D + 8 * 2 * D));
        va[s * C::NDB + b] = __builtin_bit_cast(v8h, __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    }
  };
  // P operand of a tile from its RTZ indices y = 1024 + P_i8: f16(P_i8 * sp), sp = f16(er / 127)
  auto p_operand = [&](const unsigned* y, float er, v4u* pw) {
    const _Float16 sp = (_Float16)(er * (1.0f / 127.0f));
    const v2h sp2 = {sp, sp};
    const _Float16 nsp = (_Float16)(-1024.0f) * sp;
    const v2h nsp2 = {nsp, nsp};
#pragma unroll
    for (int j = 0; j < 8; ++j)
      pw[j / 4][j % 4] =
          __builtin_bit_cast(unsigned, __builtin_elementwise_fma(__builtin_bit_cast(v2h, y[j]), sp2, nsp2));
  };

  // The softmax of S(t) (acc) beside QK(t+1) (-> sn) and PV(t-1) (P operand pp): P(t) -> pc.
  // `mfma` = false: the prologue's tile 0 (no MFMAs to interleave).
  // so_k / so_v: the ring-slot byte offsets of tiles t+1 (K) and t-1 (V)
  auto step_body = [&](int t, int so_k, int so_v, const v16i& acc, v16i& sn, const v4u* pp, v4u* pc,
                       bool mfma) {
    // this tile's scale was read one step ahead; read the next one (first: LDS reads return in
    // order, and its consumer is the next step)
    const float ck = ck_cur;
    ck_cur = ck_lds[min(t + 1, nt - 1)];
    v4i kf[C::NKS];
    v8h va[2 * C::NDB];
    if (mfma) {
      if (QA_F2_ABL & 4) {
#pragma unroll
        for (int s = 0; s < C::NKS; ++s) kf[s] = qf[s];
      } else {
        qk_load(so_k, kf);   // (t + 1 = nt: the clamped duplicate in its slot; S(nt) is never used)
      }
      if (QA_F2_ABL & 2) {
#pragma unroll
        for (int i = 0; i < 2 * C::NDB; ++i) va[i] = __builtin_bit_cast(v8h, qf[i % C::NKS]);
      } else {
        pv_load(so_v, va);
      }
    }
    // G0: row max of S(t) over the tile (both key halves), the scale
    int mx = max(max(acc[0], acc[1]), acc[2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) mx = max(max(mx, acc[r]), acc[r + 1]);
    mx = max(mx, acc[15]);
    {
      auto r = __builtin_amdgcn_permlane32_swap((unsigned)mx, (unsigned)mx, false, false);
      mx = max((int)r[0], (int)r[1]);
    }
    const float c = kmag_scale(cq * ck);
    const float nb = -KMAG * c;
#if QA_F2_S_PK
    // S = f16(f32(X c)): one v_pk_fma_f32 + one v_cvt_pk_f16_f32 per pair (common.h
    // biased_to_f16x16; the row max rounds the same way, so rm = max S)
    const _Float16 rm = biased_to_f16(mx, c, nb);
    const v2f_ c2 = {c, c}, n2 = {nb, nb};
    unsigned s2u[8];
    auto s_pairs = [&](int j0) {
#pragma unroll
      for (int j = j0; j < j0 + 4; ++j) {
        const v2f_ a = {__int_as_float(acc[2 * j]), __int_as_float(acc[2 * j + 1])};
        s2u[j] = __builtin_bit_cast(unsigned, __builtin_convertvector(__builtin_elementwise_fma(a, c2, n2), v2h));
      }
    };
#else
    const _Float16 rm = fma_mix1(__int_as_float(mx), c, nb);
    unsigned s2u[8];
#endif
    QA_F2_FENCE();
    v16i s1 = kmag;
    if (mfma) s1 = mfma_i8(kf[0], qf[0], kmag);
#if QA_F2_S_PK
    s_pairs(0);
#else
    mix8_lo(acc, c, nb, mx, s2u);
#endif
    QA_F2_FENCE();
    if (mfma) o[0] = mfma_f16(va[0], __builtin_bit_cast(v8h, pp[0]), o[0]);
#if QA_F2_S_PK
    s_pairs(4);
#else
    mix8_hi(acc, c, nb, s2u);
#endif
    QA_F2_FENCE();
    if (mfma && C::NKS > 1) s1 = mfma_i8(kf[1], qf[1], s1);
    v2h d[8];
    const v2h rm2 = {rm, rm};
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = __builtin_bit_cast(v2h, s2u[j]) - rm2;   // f16(S - rm)
    QA_F2_FENCE();
    if (mfma) o[1] = mfma_f16(va[1], __builtin_bit_cast(v8h, pp[0]), o[1]);
    v2h e[8];
    exp2_pk4(&d[0], &e[0]);
    QA_F2_FENCE();
    if (mfma && C::NKS > 2) s1 = mfma_i8(kf[2], qf[2], s1);
    exp2_pk4(&d[4], &e[4]);
    QA_F2_FENCE();
    if (mfma && C::NDB > 2) o[2] = mfma_f16(va[2], __builtin_bit_cast(v8h, pp[0]), o[2]);
    const v2h es = ((e[0] + e[1]) + (e[2] + e[3])) + ((e[4] + e[5]) + (e[6] + e[7]));
    QA_F2_FENCE();
    if (mfma && C::NKS > 3) s1 = mfma_i8(kf[3], qf[3], s1);
    const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
    unsigned y[8];
    p_index8(e, k127, y);   // y = 1024 + trunc(127 e) (RTZ around the 8 ops)
    QA_F2_FENCE();
    if (mfma && C::NDB > 3) o[3] = mfma_f16(va[3], __builtin_bit_cast(v8h, pp[0]), o[3]);
    // the P operand with the current reference m (recomputed below if m moves)
    const float er = exp2_f32((float)(_Float16)(rm - m));
    QA_F2_FENCE();
    if (mfma) o[0] = mfma_f16(va[C::NDB + 0], __builtin_bit_cast(v8h, pp[1]), o[0]);
    p_operand(y, er, pc);
    QA_F2_FENCE();
    if (mfma) o[1] = mfma_f16(va[C::NDB + 1], __builtin_bit_cast(v8h, pp[1]), o[1]);
    const float hs = pk_hsum(es);
    const float l_prev = l;
    l = fmaf(hs, er, l);
    QA_F2_FENCE();
    if (mfma && C::NDB > 2) o[2] = mfma_f16(va[C::NDB + 2], __builtin_bit_cast(v8h, pp[1]), o[2]);
    const bool move = __ballot((float)rm > mthr) != 0;
    // (materialised here, beside the last MFMAs, not sunk into the branch's fall-through)
    asm volatile("" : "+v"(pc[0]), "+v"(pc[1]), "+v"(l));
    QA_F2_FENCE();
    if (mfma && C::NDB > 3) o[3] = mfma_f16(va[C::NDB + 3], __builtin_bit_cast(v8h, pp[1]), o[3]);
    sn = s1;
    if (move) {
      // (the empty volatile asm keeps this rare branch a branch)
      asm volatile("" ::: "memory");
      const _Float16 nm = m > rm ? m : rm;
      const float r = exp2_f32((float)(_Float16)(m - nm));
      m = nm;
      mthr = (float)m + C::THR;
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) o[b] *= r;
      const float er2 = exp2_f32((float)(_Float16)(rm - m));
      l = fmaf(hs, er2, l_prev * r);
      p_operand(y, er2, pc);
    }
  };
  auto pv_last = [&](int so, const v4u* pp) {
    v8h va[2 * C::NDB];
    pv_load(so, va);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < C::NDB; ++b)
        o[b] = mfma_f16(va[s * C::NDB + b], __builtin_bit_cast(v8h, pp[s]), o[b]);
  };

  vmem_drain();   // tiles 0..3 landed
  __syncthreads();

  v16i sa, sb;
  v4u pa[2], pb[2];
  if (active) {
    v4i kf[C::NKS];
    qk_load(slot_off(0), kf);
    sa = kmag;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) sa = mfma_i8(kf[s], qf[s], sa);
    qk_load(slot_off(1), kf);   // (nt = 1: the clamped duplicate)
    sb = kmag;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) sb = mfma_i8(kf[s], qf[s], sb);
    ck_cur = ck_lds[0];
    v16i unused;
    step_body(0, 0, 0, sa, unused, pb, pa, false);
  }
  // step t: tile t+1 landed (t+2 may be in flight); every wave is past step t-1, so the slot of tile
  // t-2 is free for tile t+3.  The slot offsets of tiles t+1 (K), t-1 (V) and t+3 (DMA) rotate in
  // SGPRs (no modulo per step).
  int so_k = 2 * C::SLOT, so_v = 0, so_d = 4 * C::SLOT;
  auto rot = [](int x) { x += C::SLOT; return (int)__builtin_amdgcn_readfirstlane(x == NS * C::SLOT ? 0 : x); };
  auto step = [&](int t, const v16i& acc, v16i& sn, const v4u* pp, v4u* pc) {
    if (QA_F2_ABL & 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(C::IPW) : "memory");
    else ring_wait_barrier<C::IPW>();
    if (!(QA_F2_ABL & 8)) dma.issue(smem_lds + so_d, min(t + 3, nt - 1));
    if (active) step_body(t, so_k, so_v, acc, sn, pp, pc, true);
    so_k = rot(so_k);
    so_v = rot(so_v);
    so_d = rot(so_d);
  };
  int t = 1;
  for (; t + 1 < nt; t += 2) {
    step(t, sb, sa, pa, pb);       // S(t) in sb, P(t-1) in pa -> S(t+1) in sa, P(t) in pb
    step(t + 1, sa, sb, pb, pa);   // S(t+1) in sa, P(t) in pb -> S(t+2) in sb, P(t+1) in pa
  }
  if (t < nt) {
    step(t, sb, sa, pa, pb);
    if (active) pv_last(slot_off(nt - 1), pb);
  } else if (active) {
    pv_last(slot_off(nt - 1), pa);
  }
  vmcnt_wait_all();
  __syncthreads();   // the ring becomes the output staging area

  if (!active) return;
  // epilogue: lse = fp16(m + fp16(log2 l)); O = fp16(O / l)   (int8:252-257)
  l = pair_sum(l);
  const long qrow = head_row0 + q0 + c32;
  if (h == 0) lse[qrow] = (_Float16)((float)m + (float)(_Float16)log2_f32(l));
  const float inv = 1.0f / l;
  store_rows<D, _Float16, 1, false>(o, inv, smem + wave * RowTile<D, _Float16>::BYTES,
                                    out + (head_row0 + q0) * D, lane);
}

template <int D>
static int launch_fwd_f2(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                         const void* vdq, void* out, void* lse, long bh, long sq_tok, long sk_tok,
                         int group, float qks, hipStream_t st) {
  using C = Int8FwdCfg<D, PV_F16>;
  const int nq = (int)((sq_tok + C::QROWS - 1) / C::QROWS);
  const int lds = F2Cfg<D>::RING + (int)(((sk_tok / 32) * 4 + 15) / 16 * 16);
  { static int granted_ = 0; if (!lds_grant((const void*)int8_attn_fwd_f2_kernel<D>, lds, granted_)) return 1; }
  hipLaunchKernelGGL((int8_attn_fwd_f2_kernel<D>), dim3((unsigned)(nq * bh)), dim3(256), lds, st,
                     (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,
                     (const _Float16*)vdq, (_Float16*)out, (_Float16*)lse, (int)bh, (int)sq_tok,
                     (int)sk_tok, group, qks);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace qattn

using namespace qattn;

// The PV_F16 forward (qattn_int8_attn_fwd_ex's operands: the quantiser's f16 vdq image) on the
// two-tile pipeline; non-causal only.  Returns 1 for what it does not cover (causal, head_dim other
// than 64 / 128, token counts not multiples of 32, a key count whose scale table does not fit LDS).
extern "C" int qattn_int8_attn_fwd_f2(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                                      const void* vdq, void* out, void* lse, long bh, long sq_tok,
                                      long sk_tok, int group, int head_dim, float qks, void* stream) {
  if (sq_tok % 32 != 0 || sk_tok % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq_tok == 0) return 0;
  if (sk_tok == 0) return 1;
  // grouped heads with short query blocks run as one virtual head per group (int8_attn_fwd.hip)
  if (group > 1 && sq_tok % Int8FwdCfg<128, PV_F16>::QROWS != 0) {
    sq_tok *= group;
    bh /= group;
    group = 1;
  }
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    return launch_fwd_f2<128>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, sq_tok, sk_tok, group, qks, st);
  return launch_fwd_f2<64>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, sq_tok, sk_tok, group, qks, st);
}
