// Tile configuration, K / V swizzles and the LDS-DMA plan of one 32-key tile of the int8 attention
// forward (int8_attn_fwd.hip).
#pragma once
#include "common.h"

namespace qattn {

enum PvMode { PV_F16 = 0, PV_I8 = 1 };

// A/B knobs (tools/ab_build.sh, tools/ab_time.py; measured on MI355X):
//   QA_FWD_WAVES    waves (32 query rows each) per workgroup.  8 halve the L2 -> LDS bytes per
//                   query but measured 2-3 % slower than 4.
//   QA_FWD_OCC_F16  workgroups per CU of the PV_F16 kernel (3: <= 168 VGPRs, 2: <= 256).
//   QA_FWD_QK_BIAS  -1 (default): the biased S accumulator (one v_fma_mix per score) in PV_I8 (which
//                   keeps the 16-register seed for its P.V anyway), the int32 -> fp32 conversion in
//                   PV_F16 (whose 168-VGPR budget the seed would overflow into scratch); 0 / 1 force it.
#ifndef QA_FWD_WAVES
#define QA_FWD_WAVES 4
#endif
#ifndef QA_FWD_OCC_F16
#define QA_FWD_OCC_F16 3
#endif
#ifndef QA_FWD_QK_BIAS
#define QA_FWD_QK_BIAS -1
#endif
//   QA_FWD_S_PK     S = f16(X c) on the biased accumulator through v_pk_fma_f32 + v_cvt_pk_f16_f32
//                   (1, default: compiler builtins, 1-1.5 % faster, two same-box alternations) instead
//                   of v_fma_mix{lo,hi}_f16 inline asm (0); common.h biased_to_f16x16.
#ifndef QA_FWD_S_PK
#define QA_FWD_S_PK 1
#endif
//   QA_FWD_LITERAL_P  1: every tile's P_i8 by the reference's literal chain (undeferred running max,
//                   fp32 exp2, IEEE divisions), as the causal diagonal tiles always do; 0: only those.
//   QA_FWD_THR      the deferred running max moves when a row's tile max exceeds it by more than
//                   this (log2 units); 0 moves it on every increase, as the reference does.
#ifndef QA_FWD_THR
#define QA_FWD_THR 8.0f
#endif
#ifndef QA_FWD_LITERAL_P
#define QA_FWD_LITERAL_P 0
#endif

template <int D, int PV>
struct Int8FwdCfg {
  static constexpr int WAVES = QA_FWD_WAVES;
  static constexpr int QROWS = 32 * WAVES;      // query rows per workgroup
  static constexpr int KT = 32;                 // keys per tile / ring slot
  static constexpr int NSLOT = 4;               // ring slots
  static constexpr int K_BYTES = KT * D;        // int8 K tile
  static constexpr int V_BYTES = PV == PV_F16 ? KT * D * 2 : KT * D;   // f16 vdq / i8 V^T image
  static constexpr int SLOT = K_BYTES + V_BYTES;
  static constexpr int NKS = D / 32;            // i8 k-steps for QK^T
  static constexpr int NDB = D / 32;            // 32-wide d blocks of O^T
  static constexpr int K_CH = D / 16;           // 16-B chunks per K row
  static constexpr int V_CH = D * 2 / 16;       // 16-B chunks per vdq row
  static constexpr int K_SW_SHIFT = (D == 128) ? 1 : 2;
  static constexpr int V_SW_SHIFT = (D == 128) ? 2 : 1;
  static constexpr int K_INST = K_BYTES / 1024; // 1-KiB LDS-DMA wave instructions per tile
  static constexpr int V_INST = V_BYTES / 1024;
  static constexpr int INST = K_INST + V_INST;
  static constexpr int IPW = (INST + WAVES - 1) / WAVES;   // per wave, padded (counted vmcnt)
  // waves per SIMD the register budget must allow (__launch_bounds__ second argument): two (<= 256
  // VGPRs), three for the PV_F16 kernel at QA_FWD_OCC_F16 = 3 with 4-wave workgroups
  static constexpr int WPS = (PV == PV_F16 && WAVES == 4) ? QA_FWD_OCC_F16 : 2;
  static constexpr bool QK_BIAS = QA_FWD_QK_BIAS < 0 ? PV == PV_I8 : QA_FWD_QK_BIAS != 0;
  // the ring, reused as the output staging area of the epilogue
  static constexpr int STAGE = WAVES * RowTile<D, _Float16>::BYTES;
  static constexpr int RING = NSLOT * SLOT > STAGE ? NSLOT * SLOT : STAGE;
  static constexpr float THR = QA_FWD_THR;   // deferred running-max threshold (log2 units)
};

template <int D>
QA_DEVICE int k_sw(int row) {
  constexpr int K_CH = D / 16;
  return (row >> ((D == 128) ? 1 : 2)) & (K_CH - 1);
}
template <int D>
QA_DEVICE int v_sw(int row) {
  return (row & 3) << ((D == 128) ? 2 : 1);
}

// LDS-DMA plan of one 32-key tile (K rows, then the V operand), IPW instructions per wave.  Waves
// whose padded slots run past INST re-issue their first instruction (same bytes to the same place:
// benign), so every wave has exactly IPW DMAs in flight per tile and vmcnt(IPW) means "all but the
// last tile".  Per instruction: a lane-constant source byte offset (swizzle applied), a wave-uniform
// LDS offset inside the slot and the tile stride; the tile's base pointers are scalar.
//   K: row-major int8 rows, 16-B chunks XOR-swizzled by row.
//   V, PV_F16: row-major f16 vdq rows, swizzled for the transposed ds_read_b64_tr_b16 reads.
//   V, PV_I8: the vt operand image, already in MFMA-operand order: a plain 1-KiB copy per piece.
template <int D, int PV>
struct DmaPlan {
  using C = Int8FwdCfg<D, PV>;
  unsigned voff[C::IPW];
  unsigned lds_off[C::IPW];
  unsigned stride[C::IPW];
  v4u rsrc[C::IPW];
  QA_DEVICE void init(int wave, int lane, int S, const int8_t* kbase, const void* vbase) {
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
      } else if constexpr (PV == PV_F16) {
        const int vi = inst - C::K_INST;
        constexpr int RPI = 64 / C::V_CH;
        const int row = vi * RPI + lane / C::V_CH, p = lane % C::V_CH;
        voff[i] = row * 2 * D + 16 * (p ^ v_sw<D>(row));
        lds_off[i] = C::K_BYTES + vi * 1024;
        stride[i] = C::V_BYTES;
        rsrc[i] = make_rsrc(vbase, (unsigned)S * 2 * D);
      } else {   // PV_I8: the operand-order vt image, plain 1-KiB pieces
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

}  // namespace qattn
