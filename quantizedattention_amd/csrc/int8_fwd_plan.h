// Tile configuration, K / V swizzles and the LDS-DMA plan of one 32-key tile of the int8 attention
// forward (int8_attn_fwd.hip).
#pragma once
#include "common.h"
#include "exp2_corr.h"

namespace qattn {

// A/B knobs (tools/ab_build.sh, tools/ab_time.py; measured on MI355X):
//   QA_FWD_WAVES    waves (32 query rows each) per workgroup.  8 halve the L2 -> LDS bytes per
//                   query but measured 2-3 % slower than 4.
#ifndef QA_FWD_WAVES
#define QA_FWD_WAVES 4
#endif
//   QA_FWD_THR      the deferred running max moves when a row's tile max exceeds it by more than
//                   this (log2 units); 0 moves it on every increase, as the reference does.
#ifndef QA_FWD_THR
#define QA_FWD_THR 8.0f
#endif
//   QA_FWD_LIT_K    the literal-chain vote: a tile's P_i8 follows the reference's chain
//                   (undeferred running max, correctly rounded exp2, IEEE quotient) when some row of
//                   the wave has er * K > l, i.e. when the tile can weigh more than 1/K of the row's
//                   softmax sum so far; every other tile takes the fast f16 chain, whose occasional
//                   one-step P_i8 difference then moves O by at most |v| / (127 K).  0: every tile
//                   literal (priced variant), -1: only the causal diagonal tiles (round-4 behaviour).
#ifndef QA_FWD_LIT_K
#define QA_FWD_LIT_K 2
#endif
//   QA_FWD_DEFER    N > 0: the votes are taken again against the final row sums, N slots per wave
//                   (every tile takes the fast chain; the waves whose vote still holds are recomputed
//                   by a fixup launch that votes at the tile, int8_attn_fwd.hip); 0: vote at the tile.
#ifndef QA_FWD_DEFER
#define QA_FWD_DEFER 8
#endif

template <int D>
struct Int8FwdCfg {
  static constexpr int WAVES = QA_FWD_WAVES;
  static constexpr int QROWS = 32 * WAVES;      // query rows per workgroup
  static constexpr int KT = 32;                 // keys per tile / ring slot
  static constexpr int NSLOT = 4;               // ring slots
  static constexpr int K_BYTES = KT * D;        // int8 K tile
  static constexpr int V_BYTES = KT * D;        // int8 V^T operand image
  static constexpr int SLOT = K_BYTES + V_BYTES;
  static constexpr int NKS = D / 32;            // i8 k-steps for QK^T
  static constexpr int NDB = D / 32;            // 32-wide d blocks of O^T
  static constexpr int K_CH = D / 16;           // 16-B chunks per K row
  static constexpr int K_INST = K_BYTES / 1024; // 1-KiB LDS-DMA wave instructions per tile
  static constexpr int V_INST = V_BYTES / 1024;
  static constexpr int INST = K_INST + V_INST;
  static constexpr int IPW = (INST + WAVES - 1) / WAVES;   // per wave, padded (counted vmcnt)
  // the ring, reused as the output staging area of the epilogue
  static constexpr int STAGE = WAVES * RowTile<D, _Float16>::BYTES;
  static constexpr int RING = NSLOT * SLOT > STAGE ? NSLOT * SLOT : STAGE;
  static constexpr int CORR_BYTES = EXP2_CORR_WORDS * 4;   // the exp2 correction table (LDS copy)
  static constexpr float THR = QA_FWD_THR;   // deferred running-max threshold (log2 units)
  static constexpr int LIT_K = QA_FWD_LIT_K;
  static constexpr int NV = QA_FWD_DEFER > 0 ? QA_FWD_DEFER : 1;   // deferred-vote slots per wave
  static constexpr int CAND_BYTES = WAVES * NV * 128 * 4;           // {er, m} per lane and slot
  // LDS bytes of a launch over nt key tiles: ring, two per-tile scale tables (padded to 4 tiles),
  // then one region that holds the deferred votes in the fast pass and the correction table in the
  // fixup pass (the fast pass never loads the table; the inline fixup loads it after the fast pass's
  // epilogue has read its votes and the workgroup has passed a barrier)
  static constexpr int VOTE_OR_CORR = CORR_BYTES > CAND_BYTES ? CORR_BYTES : CAND_BYTES;
  static constexpr int lds_bytes(int nt) { return RING + ((nt + 3) / 4 * 4) * 8 + VOTE_OR_CORR; }
};

template <int D>
QA_DEVICE int k_sw(int row) {
  constexpr int K_CH = D / 16;
  return (row >> ((D == 128) ? 1 : 2)) & (K_CH - 1);
}

// LDS-DMA plan of one 32-key tile (K rows, then the V operand), IPW instructions per wave.  Waves
// whose padded slots run past INST re-issue their first instruction (same bytes to the same place:
// benign), so every wave has exactly IPW DMAs in flight per tile and vmcnt(IPW) means "all but the
// last tile".  Per instruction: a lane-constant source byte offset (swizzle applied), a wave-uniform
// LDS offset inside the slot and the tile stride; the tile's base pointers are scalar.
//   K: row-major int8 rows, 16-B chunks XOR-swizzled by row.
//   V: the vt operand image, already in MFMA-operand order: a plain 1-KiB copy per piece.
template <int D>
struct DmaPlan {
  using C = Int8FwdCfg<D>;
  unsigned voff[C::IPW];
  unsigned lds_off[C::IPW];
  unsigned stride[C::IPW];
  v4u rsrc[C::IPW];
  QA_DEVICE void init(int wave, int lane, int S, const int8_t* kbase, const int8_t* vbase) {
#pragma unroll
    for (int i = 0; i < C::IPW; ++i) {
      int inst = wave + C::WAVES * i;
      if (inst >= C::INST) inst = wave % C::INST;   // (more waves than pieces: re-issue one)
      if (inst < C::K_INST) {
        constexpr int RPI = 64 / C::K_CH;
        const int row = inst * RPI + lane / C::K_CH, p = lane % C::K_CH;
        voff[i] = row * D + 16 * (p ^ k_sw<D>(row));
        lds_off[i] = inst * 1024;
        stride[i] = C::K_BYTES;
        rsrc[i] = make_rsrc(kbase, (unsigned)S * D);
      } else {   // the operand-order vt image, plain 1-KiB pieces
        const int vi = inst - C::K_INST;
        voff[i] = vi * 1024 + 16 * lane;
        lds_off[i] = C::K_BYTES + vi * 1024;
        stride[i] = C::V_BYTES;
        rsrc[i] = make_rsrc(vbase, (unsigned)S * D);
      }
    }
  }
  QA_DEVICE void issue(unsigned slot_lds, int tile) const {
#pragma unroll
    for (int i = 0; i < C::IPW; ++i)
      dma16_buf(rsrc[i], voff[i], (unsigned)tile * stride[i], slot_lds + lds_off[i]);
  }
};

// exp2 correctly rounded to f32 at an fp16 argument x <= 0: v_exp_f32 corrected by the table
// (exp2_corr.h: one signed byte per argument, copied to LDS at `tab`) for -32 <= x <= 0; below -32
// v_exp_f32 as is (faithful, and such values weigh less than 2^-32 of the row).  The literal P chain
// needs the correctly rounded value: P / sp lands on 127 for a tile's maximum key up to two roundings,
// so the last ulp of exp2 decides between P_i8 = 126 and 127 (tests/test_oracle_sensitivity.py).
typedef __attribute__((address_space(3))) const signed char LdsI8;
QA_DEVICE float exp2_cr(_Float16 x, LdsI8* tab) {
  const float y = exp2_f32((float)x);
  const unsigned i = min((unsigned)__builtin_bit_cast(unsigned short, x) & 0x7fffu, (unsigned)EXP2_CORR_ARGS);
  return __int_as_float(__float_as_int(y) + (int)tab[i]);
}

}  // namespace qattn
