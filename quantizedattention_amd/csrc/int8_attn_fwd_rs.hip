// SageAttention-3 int8 attention forward, role-split form (replaces the attention part of
// helion_atten_int8_hl_dot_fwd, attention_int8.py:170-257), per (batch, head).
//
// Why a role split.  Per 32x32 score tile the reference recipe costs ~90 vector instructions (f16
// rounding of S, row max, exp2, P_i8 truncation, row sums; int8:197-250) beside 12 MFMAs.  A SIMD
// issues the vector instructions of all its waves through one port, and a wave that mixes MFMAs
// and vector work pays for both in its own issue stream (tools/ubench/coexec.py: two mixed waves
// take the sum of their issue times).  A wave that issues only MFMAs keeps the matrix pipe paced
// at 32 cycles per MFMA beside vector-only waves (same table: 385 cycles per 12 MFMAs with two
// vector waves beside it).  So each SIMD runs ONE matrix wave and TWO softmax waves:
//
//   matrix wave m (waves 0-3, 32 query rows each, s_setprio 2):
//     step s:  QK(s):   S^T = K_i8 . Q_i8^T (D/32 x v_mfma_i32_32x32x32_i8), S = f16(X c)
//                       (one v_fma_mix per score on the biased accumulator, common.h KMAG) -> LDS
//              PV(s-2): O^T = O^T * r + Vdq^T . P^T (2 D/32 x v_mfma_f32_32x32x16_f16)
//   softmax waves (waves 4-11; wave 4 + m + 4 h serves rows 16h..16h+15 of matrix wave m):
//     step s:  SM(s-1): S tile from LDS -> row max rm, deferred running max m (r = exp2(m_old - m)
//                       when it moves), P operand f16(P_i8 sp) -> LDS, r -> LDS, l += er sum e
//
// One workgroup barrier per step; S and P tiles are double-buffered in LDS, so the matrix waves
// compute QK(s) and PV(s-2) while the softmax waves work on tile s-1.  Numerics are those of the
// PV_F16 mode of int8_attn_fwd.hip (same P_i8 = trunc(127 exp2(f16(S - rm))), same scales, same
// deferred-max rule per softmax wave of 16 rows):  S = f16(X sq sk qks), d = f16(S - rm),
// P_i8 = trunc(127 exp2(d)), sp = f16(exp2(rm - m) / 127), O += f16(P_i8 sp) . f16(v_i8 sv),
// l += exp2(rm - m) sum exp2(d), lse = f16(m + f16(log2 l)), O = f16(O / l)  (int8:197-257).
//
// LDS (one 768-thread workgroup per CU, D = 128):
//   ring      8 slots x (K i8 4 KiB + vdq f16 8 KiB), buffer LDS-DMA by the matrix waves, 5 tiles
//             ahead; the ring becomes the output staging area of the epilogue
//   S, P      per matrix wave 2 x 2 KiB each: f16 32x32 tiles in 16-B units (query q, key group g
//             of 8 keys), unit 4q + (((q >> 2) & 3) ^ t(g)), t = {0, 3, 1, 2}: conflict-free for the
//             matrix wave's 8-B S writes and 16-B P reads and the softmax waves' 16-B S reads / P
//             writes (every ds_read_b128 lane group and ds_write_b64 16-lane group hits 16 distinct
//             4-bank quads).  Before step 1 the P area holds the Q tiles (Q DMA).
//   r         per matrix wave 2 x 32 f32: the O rescale factor of each row for the tile in flight
//   ck        sk * qks per key tile (f32), cq per matrix wave, {m, l} per row for the epilogue
#include "common.h"

// Timing-only ablations for A/B builds (tools/ab_build.sh ... -DQA_RS_ABL=n; results are wrong
// with any bit set): 1 softmax waves idle, 2 no P.V MFMAs, 4 no QK MFMAs / S conversion, 8 no K/V
// DMA, 16 softmax waves skip exp2 / P operand, 32 no s_setprio.
#ifndef QA_RS_ABL
#define QA_RS_ABL 0
#endif

namespace qattn {

// Diagnostic build only (-DQA_RS_STAMP=1, tools/rs_stamps.py): s_memtime stamps at the phase
// boundaries of steps 40..47 of workgroup 777, lanes 0 of waves 0 and NM (a matrix and a softmax
// wave), written with vector stores to a buffer of their own that no other code reads.
#ifndef QA_RS_STAMP
#define QA_RS_STAMP 0
#endif
#if QA_RS_STAMP
__device__ unsigned long long g_rs_stamp[2][8][16];
#define RS_STAMP(role, k)                                                                       \
  do {                                                                                          \
    if (blockIdx.x == 777 && s_st >= 40 && s_st < 48 && (tid & 63) == 0)                         \
      g_rs_stamp[role][s_st - 40][k] = __builtin_amdgcn_s_memtime();                            \
  } while (0)
#else
#define RS_STAMP(role, k) do { } while (0)
#endif

// MPS = matrix waves per SIMD: 1 (4 matrix + 8 softmax waves, 128 query rows per workgroup) or 2
// (8 matrix + 4 softmax waves, 256 rows: half the K/V stream per row, tools/ab_rs.py)
template <int D, int MPS>
struct RsCfg {
  static_assert(D == 128, "the role-split forward is laid out for head_dim 128");
  static_assert(MPS == 1 || MPS == 2, "one or two matrix waves per SIMD");
  static constexpr int NM = 4 * MPS;              // matrix waves
  static constexpr int NV = 4 * (3 - MPS);        // softmax waves (three waves per SIMD in all)
  static constexpr int UPV = 2 * NM / NV;         // 16-row units per softmax wave
  static constexpr int THREADS = 64 * (NM + NV);
  static constexpr int QROWS = 32 * NM;
  static constexpr int KT = 32;
  static constexpr int NKS = D / 32;              // i8 k-steps of QK^T
  static constexpr int NDB = D / 32;              // 32-wide d blocks of O^T
  static constexpr int K_BYTES = KT * D;          // K tile, i8
  static constexpr int V_BYTES = KT * D * 2;      // vdq operand image, f16
  static constexpr int SLOT = K_BYTES + V_BYTES;
  static constexpr int K_INST = K_BYTES / 1024, V_INST = V_BYTES / 1024, INST = K_INST + V_INST;
  static constexpr int DW = 4;                    // matrix waves 0..3 issue the DMA
  static constexpr int IPW = INST / DW;           // DMA pieces per issuing wave and tile
  static_assert(INST % DW == 0, "every issuing wave issues the same number of pieces");
  static constexpr int NSLOT = MPS == 1 ? 8 : 6;
  static constexpr int LOOK = NSLOT - 3;          // DMA lookahead (tiles)
  // at each step barrier tile s+2 has landed: tiles s+3 .. s+LOOK may still be in flight
  static constexpr int VMCNT = (LOOK - 2) * IPW;
  static_assert(NSLOT >= LOOK + 3, "a slot is refilled only after its V fragments were read");
  static constexpr int RING = NSLOT * SLOT;
  static constexpr int TILE = 32 * 32 * 2;        // one f16 32x32 tile
  static constexpr int S_OFF = RING;
  static constexpr int P_OFF = S_OFF + NM * 2 * TILE;
  static constexpr int R_OFF = P_OFF + NM * 2 * TILE;
  static constexpr int LM_OFF = R_OFF + NM * 2 * 32 * 4;
  static constexpr int CQ_OFF = LM_OFF + NM * 32 * 8;
  static constexpr int CK_OFF = CQ_OFF + (NM * 4 + 15) / 16 * 16;
  static constexpr float THR = 8.0f;
  static_assert(NM * RowTile<D, _Float16>::BYTES <= RING, "epilogue staging fits the ring");
  static_assert(NKS * 1024 <= 2 * TILE, "the Q tile of a matrix wave fits its P buffers");
  static int lds_bytes(long sk_tok) { return CK_OFF + (int)(((sk_tok / 32) * 4 + 15) / 16 * 16); }
};

// w = f16(P_i8 * sp) for 4 pairs: y = RTZ_f16(127 e + 1024) = P_i8 + 1024, w = RNE_f16(y sp - 1024 sp)
// (p_operand8 of common.h on 4 pairs)
QA_DEVICE void p_operand4(const v2h* e, v2h sp2, v2h nsp2, v2h* w) {
  const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
  const v2h k1024 = {(_Float16)1024.0f, (_Float16)1024.0f};
  v2h y[4];
  asm volatile(
      "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 3\n\t"
      "s_nop 1\n\t"
      "v_pk_fma_f16 %0, %4, %8, %9\n\t"
      "v_pk_fma_f16 %1, %5, %8, %9\n\t"
      "v_pk_fma_f16 %2, %6, %8, %9\n\t"
      "v_pk_fma_f16 %3, %7, %8, %9\n\t"
      "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 0\n\t"
      "s_nop 1"
      : "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3])
      : "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(e[3]), "v"(k127), "v"(k1024));
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = __builtin_elementwise_fma(y[j], sp2, nsp2);
}

QA_DEVICE void rs_barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS-DMA plan of one tile over the four matrix waves (IPW pieces each, 1 KiB per piece):
//   K pieces p < K_INST: the tile in A-operand order, chunk-major: LDS unit 32 c + row (16 B) holds
//     K[row][16c .. +16] (c = 2 s + h: the k-step s half h), so piece p lane l <- row l & 31,
//     chunk 2p + (l >> 5), and the K fragment of lane l for k-step s is at 1024 s + 16 l;
//   V pieces: a plain 1-KiB copy of the vdq operand image (qattn_int8_quant_vop), piece 4 s2 + b at
//     K_BYTES + 1024 (4 s2 + b), lane l at + 16 l.
template <int D, int MPS>
struct RsDma {
  using C = RsCfg<D, MPS>;
  unsigned voff[C::IPW];
  unsigned lds_off[C::IPW];
  v4u krs, vrs;
  QA_DEVICE void init(int mw, int lane, int Sk, const int8_t* kbase, const _Float16* vbase) {
    krs = make_rsrc(kbase, (unsigned)Sk * D);
    vrs = make_rsrc(vbase, (unsigned)Sk * D * 2);
#pragma unroll
    for (int i = 0; i < C::IPW; ++i) {
      const int inst = mw + C::DW * i;
      if (inst < C::K_INST) {
        voff[i] = (unsigned)((lane & 31) * D + 32 * inst + 16 * (lane >> 5));
        lds_off[i] = 1024u * inst;
      } else {
        voff[i] = (unsigned)(1024 * (inst - C::K_INST) + 16 * lane);
        lds_off[i] = (unsigned)(C::K_BYTES + 1024 * (inst - C::K_INST));
      }
    }
  }
  QA_DEVICE void issue(unsigned slot_lds, int tile, int mw) const {
#pragma unroll
    for (int i = 0; i < C::IPW; ++i) {
      const bool is_k = mw + C::DW * i < C::K_INST;   // (wave-uniform)
      dma16_buf(is_k ? krs : vrs, voff[i], (unsigned)tile * (is_k ? C::K_BYTES : C::V_BYTES),
                slot_lds + lds_off[i]);
    }
  }
};

template <int D, int MPS>
__global__ __launch_bounds__((RsCfg<D, MPS>::THREADS), 3) void int8_attn_fwd_rs_kernel(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const _Float16* __restrict__ vop, _Float16* __restrict__ out,
    _Float16* __restrict__ lse, int BH, int Sq, int Sk, int G, float qks) {
  using C = RsCfg<D, MPS>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* ck_lds = reinterpret_cast<float*>(smem + C::CK_OFF);
  float* cq_lds = reinterpret_cast<float*>(smem + C::CQ_OFF);

  const int nq = (Sq + C::QROWS - 1) / C::QROWS;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int nt = Sk / C::KT;
  const long kv_row0 = (long)(bh / G) * Sk;
  const long head_row0 = (long)bh * Sq;

  if (wave < C::NM) {
    // ================================================================ matrix wave
    if (!(QA_RS_ABL & 32)) __builtin_amdgcn_s_setprio(2);
    const int mw = wave;
    const int h = lane >> 5, c32 = lane & 31;
    const int q0 = qt * C::QROWS + 32 * mw;
    const bool active = q0 < Sq;
    const unsigned smem_lds = lds_addr(smem);
    char* sbuf = smem + C::S_OFF + mw * 2 * C::TILE;
    const char* pbuf = smem + C::P_OFF + mw * 2 * C::TILE;
    const float* rbuf = reinterpret_cast<const float*>(smem + C::R_OFF) + mw * 64;

    // Q tile -> this wave's P buffers by LDS-DMA, in B-operand order: piece s, lane l <- row
    // q0 + (l & 31), bytes 32 s + 16 (l >> 5) .. +16 (one ds_read_b128 per k-step reads it back)
    if (active) {
      const v4u qr = make_rsrc(q_i8 + (head_row0 + q0) * D, 32u * D);
#pragma unroll
      for (int s = 0; s < C::NKS; ++s)
        dma16_buf(qr, (unsigned)(c32 * D + 32 * s + 16 * h), 0u, lds_addr(pbuf) + (unsigned)(1024 * s));
    }
    const bool dw = mw < C::DW;   // (wave-uniform) this wave issues DMA pieces
    RsDma<D, MPS> dma;
    dma.init(mw & (C::DW - 1), lane, Sk, k_i8 + kv_row0 * D, vop + kv_row0 * D);
    if (dw) {
#pragma unroll
      for (int i = 0; i < C::LOOK; ++i)
        dma.issue(smem_lds + (i % C::NSLOT) * C::SLOT, min(i, nt - 1), mw);
    }

    // The biased-accumulator seed (common.h KMAG) is written into the S accumulator at the end of
    // every step, 8 v_mov_b64 from an SGPR pair: a 16-register seed held beside the accumulator would
    // push the wave past its 168-register budget.  (An asm VALU write feeding an MFMA operand: the
    // step's DMA issue, s_waitcnt and s_barrier lie between it and the next QK MFMA.)
    const unsigned long kmag2 = 0x4B4000004B400000ul;
    auto kmag_seed = [&](v16i& z) {
      unsigned long p[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_mov_b64 %0, %1" : "=v"(p[i]) : "s"(kmag2));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const v2i w = __builtin_bit_cast(v2i, p[i]);
        z[2 * i] = w[0];
        z[2 * i + 1] = w[1];
      }
    };
    v16f o[C::NDB];
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};

    // lane-linear fragments: K k-step s at slot + 1024 s + 16 lane, V piece p at slot + K_BYTES +
    // 1024 p + 16 lane, P k-step s2 at pbuf + 1024 s2 + 16 lane; S: unit 32 g + c32, half h
    const int l16 = 16 * lane;
    const int soff = 16 * c32 + 8 * h;
    auto k_load = [&](int t, v4i* kf) {
      const char* kl = smem + (t % C::NSLOT) * C::SLOT + l16;
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) kf[s] = *reinterpret_cast<const v4i*>(kl + 1024 * s);
    };
    auto v_load = [&](int t, v8h* va) {
      const char* vl = smem + (t % C::NSLOT) * C::SLOT + C::K_BYTES + l16;
#pragma unroll
      for (int p = 0; p < 2 * C::NDB; ++p) va[p] = *reinterpret_cast<const v8h*>(vl + 1024 * p);
    };

    v16i sacc;
    kmag_seed(sacc);
    // tiles 0 and 1 and the Q tile have landed (vmcnt: the DMA waves' Q pieces are older than their
    // tile pieces; the other matrix waves issued only their Q pieces), the softmax waves have staged
    // ck / cq
    if (dw) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(C::VMCNT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

    v4i qf[C::NKS];
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v4i*>(pbuf + 1024 * s + l16);
    const float cq = cq_lds[mw];
    v4i kf[C::NKS];
    k_load(0, kf);
    v8h va[2 * C::NDB];

    // one step: QK(s) (if qk), PV(s-2) (if pv); then S(s) -> LDS and the K(s+1) / V(s-1) fragments
    // for the next step.  A matrix wave past the last query row (active false) computes on whatever
    // its buffers hold: nothing reads its S tiles (its softmax waves idle) and its O is not stored.
    auto step = [&](int s, bool qk, bool pv, bool pre_k, bool pre_v) {
      [[maybe_unused]] const int s_st = wave == 0 ? s : -1;
      RS_STAMP(0, 0);
      if (qk && !(QA_RS_ABL & 4)) {
        sacc = mfma_i8(kf[0], qf[0], sacc);
#pragma unroll
        for (int ks = 1; ks < C::NKS; ++ks) sacc = mfma_i8(kf[ks], qf[ks], sacc);
      }
      __builtin_amdgcn_sched_barrier(0);
      RS_STAMP(0, 1);
      if (pv) {
        const char* pb = pbuf + (s & 1) * C::TILE + l16;   // P(s-2): buffer (s-2) & 1
        const v8h p0 = *reinterpret_cast<const v8h*>(pb);
        const v8h p1 = *reinterpret_cast<const v8h*>(pb + 1024);
        const float r = rbuf[(s & 1) * 32 + c32];
        RS_STAMP(0, 2);
        if (!(QA_RS_ABL & 1) && __ballot(r != 1.0f) != 0) {
          asm volatile("" ::: "memory");   // (rare: keep it a branch)
#pragma unroll
          for (int b = 0; b < C::NDB; ++b) o[b] *= r;
        }
        if (!(QA_RS_ABL & 2)) {
#pragma unroll
          for (int b = 0; b < C::NDB; ++b) o[b] = mfma_f16(va[b], p0, o[b]);
#pragma unroll
          for (int b = 0; b < C::NDB; ++b) o[b] = mfma_f16(va[C::NDB + b], p1, o[b]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      RS_STAMP(0, 3);
      if (qk && !(QA_RS_ABL & 4)) {
        // S = f16(X c), c = sq sk qks (int8:200-203), on the biased accumulator
        const float c = kmag_scale(cq * ck_lds[s]);
        const float nb = -KMAG * c;
        const int dep = sacc[0] ^ sacc[15];   // a compiler-visible read of the MFMA result
        v2h s2[8];
        fma_mix16_after(sacc, c, nb, dep, s2);
        char* sb = sbuf + (s & 1) * C::TILE + soff;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<v2u*>(sb + 512 * g) =
              v2u{__builtin_bit_cast(unsigned, s2[2 * g]), __builtin_bit_cast(unsigned, s2[2 * g + 1])};
      }
      // the S tile must be in LDS before the barrier; the fragment prefetches for the next step need
      // not: they stay in flight across it (the compiler waits for them where they are used, and
      // their ring slots are refilled only steps later)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      RS_STAMP(0, 4);
      if (pre_k) k_load(s + 1, kf);
      if (pre_v) v_load(s - 1, va);
      if (qk) kmag_seed(sacc);
      const int tn = s + C::LOOK;
      if (dw && !(QA_RS_ABL & 8)) dma.issue(smem_lds + (tn % C::NSLOT) * C::SLOT, min(tn, nt - 1), mw);
      RS_STAMP(0, 5);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::VMCNT) : "memory");
      RS_STAMP(0, 6);
      asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };

    // steps 0 .. nt+1: QK(s) for s < nt, PV(s-2) for s >= 2
    for (int s = 0; s < 2; ++s) step(s, s < nt, false, s + 1 < nt, s == 1);
    for (int s = 2; s < nt - 1; ++s) step(s, true, true, true, true);   // steady state
    for (int s = max(2, nt - 1); s < nt + 2; ++s) step(s, s < nt, true, s + 1 < nt, s <= nt);

    // epilogue: the softmax waves publish {m, l}; every DMA of this wave has landed before the
    // barrier, so after it the ring is the output staging area
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (!active) return;
    const float2 ml = reinterpret_cast<const float2*>(smem + C::LM_OFF)[mw * 32 + c32];
    const long qrow = head_row0 + q0 + c32;
    if (h == 0) lse[qrow] = (_Float16)(ml.x + (float)(_Float16)log2_f32(ml.y));
    store_rows<D, _Float16>(o, 1.0f / ml.y, smem + mw * RowTile<D, _Float16>::BYTES,
                            out + (head_row0 + q0) * D, lane);
  } else {
    // ================================================================ softmax wave
    // UPV units of 16 rows: MPS 1, wave 4 + v serves rows 16 (v >> 2) .. +16 of matrix wave v & 3;
    // MPS 2, wave 8 + v serves both halves of matrix waves v and v + 4 (the waves of its SIMD).
    // Lane l of a unit: row q = 16 half + (l & 15) of its matrix wave, keys 8g .. 8g+7 (g = l >> 4).
    const int vw = wave - C::NM;
    const int ql = lane & 15, g = lane >> 4;
    int mwu[C::UPV], qu[C::UPV];
#pragma unroll
    for (int u = 0; u < C::UPV; ++u) {
      if constexpr (MPS == 1) {
        mwu[u] = vw & 3;
        qu[u] = 16 * (vw >> 2) + ql;
      } else {
        mwu[u] = vw + 4 * (u >> 1);
        qu[u] = 16 * (u & 1) + ql;
      }
    }
    bool act[C::UPV];
    const char* sbu[C::UPV];
    char* pbu[C::UPV];
    float* rbu[C::UPV];
#pragma unroll
    for (int u = 0; u < C::UPV; ++u) {
      act[u] = qt * C::QROWS + 32 * mwu[u] < Sq;
      sbu[u] = smem + C::S_OFF + mwu[u] * 2 * C::TILE + 16 * (32 * g + qu[u]);   // unit (q, g)
      pbu[u] = smem + C::P_OFF + mwu[u] * 2 * C::TILE + 16 * (32 * g + qu[u]);
      rbu[u] = reinterpret_cast<float*>(smem + C::R_OFF) + mwu[u] * 64 + qu[u];
    }
    // (MPS 2: a workgroup's units are all active or all idle but the last partial one's)
    bool any_act = false;
#pragma unroll
    for (int u = 0; u < C::UPV; ++u) any_act = any_act || act[u];

    // stage the per-tile scales ck = sk qks and the matrix waves' cq (plain loads: the softmax waves
    // issue no LDS-DMA, so the compiler's own waits are exact here)
    for (int i = tid - 64 * C::NM; i < nt; i += 64 * C::NV) ck_lds[i] = (float)sk[kv_row0 / 32 + i] * qks;
    if (tid - 64 * C::NM < C::NM) {
      const int m2 = tid - 64 * C::NM;
      const int qb = qt * C::QROWS + 32 * m2;
      cq_lds[m2] = qb < Sq ? (float)sq[(head_row0 + qb) / 32] : 0.f;
    }
    rs_barrier_lds();

    _Float16 m[C::UPV];
    float l[C::UPV];   // this lane's keys (8g..8g+7 of every tile); the 4 lanes of a row sum at the end
#pragma unroll
    for (int u = 0; u < C::UPV; ++u) {
      m[u] = (_Float16)(-INFINITY);
      l[u] = 0.f;
    }
    // one tile of every unit, phase by phase over the units (independent chains side by side)
    auto sm = [&](int j) {
      [[maybe_unused]] const int s_st = wave == C::NM ? j + 1 : -1;
      RS_STAMP(1, 0);
      const int jb = (j & 1) * C::TILE;
      v2h x[C::UPV][4];
#pragma unroll
      for (int u = 0; u < C::UPV; ++u) {
        const v4u xs = *reinterpret_cast<const v4u*>(sbu[u] + jb);
        // (through a scalar: hipcc 7.2 folds __builtin_bit_cast of an ext-vector ELEMENT lvalue to
        // element 0 whatever the index)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const unsigned w = xs[i];
          x[u][i] = __builtin_bit_cast(v2h, w);
        }
      }
      // row max over the tile: 8 values here, then the lanes ql, ql+16, ql+32, ql+48
      v2h rm2[C::UPV];
#pragma unroll
      for (int u = 0; u < C::UPV; ++u)
        rm2[u] = __builtin_elementwise_max(__builtin_elementwise_max(x[u][0], x[u][1]),
                                           __builtin_elementwise_max(x[u][2], x[u][3]));
#pragma unroll
      for (int u = 0; u < C::UPV; ++u) {
        const unsigned w = __builtin_bit_cast(unsigned, rm2[u]);
        const auto r16 = __builtin_amdgcn_permlane16_swap(w, w, false, false);
        rm2[u] = __builtin_elementwise_max(__builtin_bit_cast(v2h, (unsigned)r16[0]),
                                           __builtin_bit_cast(v2h, (unsigned)r16[1]));
      }
#pragma unroll
      for (int u = 0; u < C::UPV; ++u) {
        const unsigned w = __builtin_bit_cast(unsigned, rm2[u]);
        const auto r32 = __builtin_amdgcn_permlane32_swap(w, w, false, false);
        rm2[u] = __builtin_elementwise_max(__builtin_bit_cast(v2h, (unsigned)r32[0]),
                                           __builtin_bit_cast(v2h, (unsigned)r32[1]));
        rm2[u] = __builtin_elementwise_max(rm2[u], __builtin_shufflevector(rm2[u], rm2[u], 1, 0));
      }
      RS_STAMP(1, 1);
      // deferred running max per unit (16 rows): moves only when a row's tile max passes m + THR
      float rout[C::UPV];
      bool mv = false;
#pragma unroll
      for (int u = 0; u < C::UPV; ++u) {
        rout[u] = 1.0f;
        mv = mv || ((float)rm2[u][0] > (float)m[u] + C::THR);
      }
      if (__ballot(mv) != 0) {
        asm volatile("" ::: "memory");   // (rare: keep it a branch)
#pragma unroll
        for (int u = 0; u < C::UPV; ++u) {
          const _Float16 rm = rm2[u][0];
          if (__ballot((float)rm > (float)m[u] + C::THR) != 0) {
            const _Float16 nm = m[u] > rm ? m[u] : rm;
            const float r = exp2_f32((float)(_Float16)(m[u] - nm));
            m[u] = nm;
            l[u] *= r;
            rout[u] = r;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < C::UPV; ++u) rbu[u][(j & 1) * 32] = rout[u];
      v2h w[C::UPV][4];
#pragma unroll
      for (int u = 0; u < C::UPV; ++u) {
        const float er = exp2_f32((float)(_Float16)(rm2[u][0] - m[u]));
        const _Float16 sp = (_Float16)(er * (1.0f / 127.0f));
        const v2h sp2 = {sp, sp};
        const v2h nsp2 = sp2 * (v2h){(_Float16)(-1024.0f), (_Float16)(-1024.0f)};
        v2h d[4], e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = x[u][i] - rm2[u];   // f16(S - rm)  (int8:211, 232-236)
        if (QA_RS_ABL & 16) {
#pragma unroll
          for (int i = 0; i < 4; ++i) w[u][i] = d[i] * sp2;
        } else {
          exp2_pk4(d, e);
          l[u] = fmaf(pk_hsum((e[0] + e[1]) + (e[2] + e[3])), er, l[u]);
          p_operand4(e, sp2, nsp2, w[u]);
        }
      }
      RS_STAMP(1, 2);
#pragma unroll
      for (int u = 0; u < C::UPV; ++u)
        *reinterpret_cast<v4u*>(pbu[u] + jb) =
            v4u{__builtin_bit_cast(unsigned, w[u][0]), __builtin_bit_cast(unsigned, w[u][1]),
                __builtin_bit_cast(unsigned, w[u][2]), __builtin_bit_cast(unsigned, w[u][3])};
    };
    rs_barrier_lds();   // step 0
    for (int j = 0; j < nt; ++j) {   // step j + 1
      if (any_act && !(QA_RS_ABL & 1)) sm(j);
      {
        [[maybe_unused]] const int s_st = wave == C::NM ? j + 1 : -1;
        RS_STAMP(1, 3);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        RS_STAMP(1, 4);
        asm volatile("s_barrier" ::: "memory");
        RS_STAMP(1, 5);
      }
    }
    rs_barrier_lds();   // step nt + 1
    // {m, l} of each row: the four lanes of row q hold partial sums over their key groups
#pragma unroll
    for (int u = 0; u < C::UPV; ++u) {
      const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(l[u]), __float_as_uint(l[u]), false, false);
      const float l2 = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
      const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(l2), __float_as_uint(l2), false, false);
      const float lt = __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
      if (g == 0 && act[u])
        reinterpret_cast<float2*>(smem + C::LM_OFF)[mwu[u] * 32 + qu[u]] = float2{(float)m[u], lt};
    }
    rs_barrier_lds();
  }
}

template <int D, int MPS>
static int launch_fwd_rs(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                         const void* vop, void* out, void* lse, long bh, long sq_tok, long sk_tok,
                         int group, float qks, hipStream_t st) {
  using C = RsCfg<D, MPS>;
  const int nq = (int)((sq_tok + C::QROWS - 1) / C::QROWS);
  const int lds = C::lds_bytes(sk_tok);
  static int granted = 0;
  if (!lds_grant((const void*)int8_attn_fwd_rs_kernel<D, MPS>, lds, granted)) return 2;
  hipLaunchKernelGGL((int8_attn_fwd_rs_kernel<D, MPS>), dim3((unsigned)(nq * bh)), dim3(C::THREADS), lds,
                     st, (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,
                     (const _Float16*)vop, (_Float16*)out, (_Float16*)lse, (int)bh, (int)sq_tok,
                     (int)sk_tok, group, qks);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace qattn

using namespace qattn;

// Matrix waves per SIMD of the default role-split form (A/B: -DQA_RS_MPS=1)
#ifndef QA_RS_MPS
#define QA_RS_MPS 2
#endif
// Largest key count the role-split forward takes (its per-tile scales sit in LDS).
static constexpr long RS_MAX_SK = (163840 - RsCfg<128, QA_RS_MPS>::CK_OFF) / 4 * 32;

extern "C" int qattn_int8_attn_fwd_rs(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                                      const void* vop, void* out, void* lse, long bh, long sq_tok,
                                      long sk_tok, int group, int head_dim, float qks, void* stream) {
  if (sq_tok % 32 != 0 || sk_tok % 32 != 0 || group < 1 || bh % group != 0 || head_dim != 128 ||
      sk_tok > RS_MAX_SK)
    return 1;
  if (bh == 0 || sq_tok == 0) return 0;
  if (sk_tok == 0) return 1;
  return launch_fwd_rs<128, QA_RS_MPS>(q_i8, sq, k_i8, sk, vop, out, lse, bh, sq_tok, sk_tok, group, qks,
                                       (hipStream_t)stream);
}

#if QA_RS_STAMP
extern "C" int qattn_rs_stamps(void* host_dst) {
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(qattn::g_rs_stamp), sizeof(qattn::g_rs_stamp)) == hipSuccess ? 0 : 2;
}
#endif
