// SageAttention-3 int8 attention forward for gfx950 (replaces the attention part of
// helion_atten_int8_hl_dot_fwd, attention_int8.py:170-257), per (batch, head).
//
// Work decomposition
//   * one workgroup = 4 waves = 128 query rows of one (b,h); wave w owns rows 32w..32w+31 = one
//     32-token q-quant block (one sq scale per wave).  3 workgroups per CU (<= 168 VGPRs).
//   * keys stream in 32-key tiles (= one Bkv block) through a 4-slot LDS ring filled by LDS-DMA
//     (global_load_lds_dwordx4: no staging registers; the bank swizzle is applied to the per-lane
//     source address, the LDS image is written lane-linearly).  One barrier per tile; the DMA of
//     tile t+3 is issued right after the barrier of tile t (two tiles of latency cover).
//   * every sk scale of the head sits in LDS (loaded once); workgroups of one head share an XCD.
//
// Per 32-key tile and wave (swapped orientation: keys in registers, query on the lane pair l, l^32),
// software-pipelined by one tile so that each wave has MFMA work beside its softmax VALU:
//     QK(t+1)   S^T = K_i8 . Q_i8^T            D/32 x v_mfma_i32_32x32x32_i8
//     SM2(t)    e = exp2(d), l, P operand        (VALU, beside the QK(t+1) MFMAs)
//     PV(t)     O^T += Vdq^T . P^T               2*D/32 x v_mfma_f32_32x32x16_f16
//     SM1(t+1)  d = S - rowmax, deferred max     (VALU, beside the PV(t) MFMAs)
// Reference rounding points (int8:197-257), with S never materialised:
//     S  = f16(acc * c)          (one v_fma_mix per element: exact product, one f16 rounding)
//     rm = f16(max_k(acc) * c)   (c = sq*sk*qks > 0: the row max commutes with the monotone scaling)
//     d  = f16(S - rm)           (S is rounded to f16 first, as the reference does: rounding
//                                 acc*c - rm once instead changes trunc(127 e) for many scores)
//     e  = exp2(d);  P_i8 = trunc(127 e);  operand = f16(P_i8 * sp),  sp = exp2(rm - m)/127
//     P_i8 + 1024 = (127 e + 1024) rounded toward zero (f16 spacing 1 in [1024, 2048)); the operand
//     is then one fma  f16((P_i8 + 1024)*sp - 1024*sp)  -> 2 packed ops per element pair.
//     l += exp2(rm - m) * sum e (fp32);  O *= exp2(m_old - m) when the running max moves.
// Vdq = fp16(v_i8 * sv) is written by the quantiser, so the fp32 accumulation of
// sum_t sp*sv*(P_i8 . v_i8) (int8:249-250) runs inside the MFMA, exact up to the fp16 rounding of
// the two dequantised operands.
// Deferred max (cdna_hip_programming.md T13): the running max m moves only when some row's tile max
// exceeds it by more than THR = 8 (log2 units); P_i8 depends only on S - rowmax(tile), O and l share
// the (possibly stale) reference, so O / l is unchanged up to rounding and operands stay <= 2^8.
#include <climits>
#include <type_traits>

#include "common.h"

namespace qattn {

#ifndef QA_FWD_OCC
#define QA_FWD_OCC 3
#endif
#ifndef QA_FWD_UNROLL
#define QA_FWD_UNROLL 0
#endif

template <int D>
struct Int8FwdCfg {
  static constexpr int WAVES = 4;
  static constexpr int QROWS = 32 * WAVES;      // query rows per workgroup
  static constexpr int KT = 32;                 // keys per tile / ring slot
  static constexpr int NSLOT = 4;               // ring slots
  static constexpr int K_BYTES = KT * D;        // int8 K tile
  static constexpr int V_BYTES = KT * D * 2;    // fp16 Vdq tile
  static constexpr int SLOT = K_BYTES + V_BYTES;
  static constexpr int NKS = D / 32;            // i8 k-steps for QK^T
  static constexpr int NDB = D / 32;            // 32-wide d blocks of O^T
  static constexpr int K_CH = D / 16;           // 16-B chunks per K row
  static constexpr int V_CH = D * 2 / 16;       // 16-B chunks per V row
  static constexpr int K_SW_SHIFT = (D == 128) ? 1 : 2;
  static constexpr int V_SW_SHIFT = (D == 128) ? 2 : 1;
  static constexpr int K_INST = K_BYTES / 1024; // 1-KiB LDS-DMA wave instructions per tile
  static constexpr int V_INST = V_BYTES / 1024;
  static constexpr int INST = K_INST + V_INST;
  static constexpr int IPW = (INST + WAVES - 1) / WAVES;   // per wave, padded (counted vmcnt)
  static constexpr float THR = 8.0f;
};

template <int D>
QA_DEVICE int k_sw(int row) {
  using C = Int8FwdCfg<D>;
  return (row >> C::K_SW_SHIFT) & (C::K_CH - 1);
}
template <int D>
QA_DEVICE int v_sw(int row) {
  using C = Int8FwdCfg<D>;
  return (row & 3) << C::V_SW_SHIFT;
}

// LDS-DMA plan of one 32-key tile (K rows then V rows), IPW instructions per wave.  Waves whose
// padded slots run past INST re-issue their first instruction (same bytes to the same place:
// benign), so every wave has exactly IPW DMAs in flight per tile and vmcnt(IPW) means "all but the
// last tile".  Per instruction: a lane-constant source byte offset (swizzle applied), a wave-uniform
// LDS offset inside the slot and whether it reads V; the tile's base pointers are scalar.
template <int D>
struct DmaPlan {
  using C = Int8FwdCfg<D>;
  unsigned voff[C::IPW];
  unsigned lds_off[C::IPW];
  unsigned stride[C::IPW];
  v4u rsrc[C::IPW];
  QA_DEVICE void init(int wave, int lane, int S, const int8_t* kbase, const _Float16* vbase) {
#pragma unroll
    for (int i = 0; i < C::IPW; ++i) {
      int inst = wave + C::WAVES * i;
      if (inst >= C::INST) inst = wave;
      if (inst < C::K_INST) {
        constexpr int RPI = 64 / C::K_CH;
        const int row = inst * RPI + lane / C::K_CH, p = lane % C::K_CH;
        voff[i] = row * D + 16 * (p ^ k_sw<D>(row));
        lds_off[i] = inst * 1024;
        stride[i] = C::K_BYTES;
        rsrc[i] = make_rsrc(kbase, (unsigned)S * D);
      } else {
        const int vi = inst - C::K_INST;
        constexpr int RPI = 64 / C::V_CH;
        const int row = vi * RPI + lane / C::V_CH, p = lane % C::V_CH;
        voff[i] = row * 2 * D + 16 * (p ^ v_sw<D>(row));
        lds_off[i] = C::K_BYTES + vi * 1024;
        stride[i] = C::V_BYTES;
        rsrc[i] = make_rsrc(vbase, (unsigned)S * 2 * D);
      }
    }
  }
  QA_DEVICE void issue(unsigned slot_lds, int tile) const {
#pragma unroll
    for (int i = 0; i < C::IPW; ++i)
      dma16_buf(rsrc[i], voff[i], (unsigned)tile * stride[i], slot_lds + lds_off[i]);
  }
};

// (compiles to v_max3_i32).  Deliberately NOT inline asm: its inputs are MFMA results, and hipcc's
// hazard recogniser inserts the MFMA-result -> VALU wait states only for instructions it emits itself.
QA_DEVICE int imax3(int a, int b, int c) { return max(max(a, b), c); }
#if defined(QA_FWD_STAMP)
__device__ unsigned long long g_fwd_stamps[32 * 4 * 64 * 8];
__device__ unsigned long long g_fwd_wginfo[8192 * 4];
#endif

// Per-wave softmax state between the two halves of a tile.
struct SmTile {
  v2h d[8];       // f16(S - rm) for the 16 scores of this lane
  float er;       // exp2(rm - m)
  _Float16 sp;    // f16(er / 127)
};

// AB (diagnostic timing builds only, never dispatched by the API): 1 = no softmax VALU,
// 2 = no PV MFMA, 3 = no QK^T MFMA, 4 = no K/V streaming (ring slot 0 reused, no barriers),
// 5 = 4 + no softmax, 6 = 1 + half the V-operand LDS reads, 7 = 1 + half the K-operand LDS reads.
// Outputs of AB != 0 are meaningless.
// Shapes: BH = batch * query heads, Sq query and Sk key tokens per head; query head
// bh reads key/value head bh / G (grouped-query attention, G = Hq / Hkv).  CAUSAL keeps key <= query
// (top-left aligned indices); masked scores are excluded (P = 0).  The reference has neither (its
// int8 path is square, ungrouped and non-causal, int8:122-127, 344); these are extensions.
template <int D, int AB = 0, bool CAUSAL = false>
__global__ __launch_bounds__(256, QA_FWD_OCC) void int8_attn_fwd_kernel(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const _Float16* __restrict__ vdq, _Float16* __restrict__ out,
    _Float16* __restrict__ lse, int BH, int Sq, int Sk, int G, float qks) {
  using C = Int8FwdCfg<D>;
  constexpr bool STREAM = AB != 4 && AB != 5;
  constexpr bool SOFTMAX = AB != 1 && AB != 5 && AB != 6 && AB != 7;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* sk_lds = reinterpret_cast<_Float16*>(smem + C::NSLOT * C::SLOT);

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
  const long head_row0 = (long)bh * Sq;           // this head's query rows
  const long kv_row0 = (long)(bh / G) * Sk;       // its key/value head's rows
  const int8_t* kbase = k_i8 + kv_row0 * D;
  const _Float16* vbase = vdq + kv_row0 * D;
  // causal: key tiles past the workgroup's last query are masked for all of its rows
  const int nt = CAUSAL ? min(Sk / C::KT, (qt * C::QROWS + C::QROWS) / C::KT) : Sk / C::KT;

  DmaPlan<D> dma;
  dma.init(wave, lane, Sk, kbase, vbase);
  const unsigned smem_lds = lds_addr(smem);
  dma.issue(smem_lds, 0);
  if (STREAM) {
    dma.issue(smem_lds + 1 * C::SLOT, min(1, nt - 1));
    dma.issue(smem_lds + 2 * C::SLOT, min(2, nt - 1));
  }
  for (int i = tid; i < nt; i += 64 * C::WAVES) sk_lds[i] = sk[kv_row0 / 32 + i];

  // ---- Q fragment (B operand of S^T = K Q^T): lane holds Q[q0+c32][32s + 16h .. +16]
  v4i qf[C::NKS];
  float sqw = 0.f;
  if (active) {
    const int8_t* qrow = q_i8 + (head_row0 + q0 + c32) * D + 16 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v4i*>(qrow + 32 * s);
    sqw = (float)sq[(head_row0 + q0) / 32];
  }
  const float cq = sqw * qks;

  // lane-constant LDS byte offsets (the swizzles depend only on row bits fixed per lane):
  //   K A-operand chunk (2s+h) of key row c32;  V^T A-operand, d-block b: key rows 4h + (i16>>2)
  //   (+16 per k-step, +8 for the 2nd read), columns 32b + 16gg + 4(i16&3)
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
  float l = 0.f;  // per-lane partial (this lane's key half); the reference's l = 1 is wiped by r = 0

  // ring slot of a tile: a runtime tile index (slot t & 3), or, with QA_FWD_UNROLL, the slot as a
  // compile-time constant (every LDS offset becomes a lane-constant VGPR plus an immediate)
  auto slot_idx = [](auto t) -> int {
    if constexpr (std::is_integral_v<decltype(t)>) return t & 3;
    else return decltype(t)::value;
  };
  auto slot_of = [&](auto t) -> const char* { return smem + (STREAM ? slot_idx(t) : 0) * C::SLOT; };

  // S^T tile t into an int32 accumulator: fragment loads and MFMAs separately, so the K loads of
  // tile t+1 can be issued ahead of the V-operand loads of tile t
  auto qk_load = [&](auto t, v4i* kf) {
    const char* kl = slot_of(t);
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
      if (AB == 7 && s >= C::NKS / 2) kf[s] = kf[s - C::NKS / 2] + 1;   // half the K reads (timing)
      else kf[s] = *reinterpret_cast<const v4i*>(kl + koff[s]);
    }
  };
  auto qk_mma = [&](const v4i* kf) -> v16i {
    v16i acc;
    if constexpr (AB == 3) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = kf[i & 3][i >> 2] + qf[i & 3][0];
    } else {
      acc = mfma_i8(kf[0], qf[0], v16i{});
#pragma unroll
      for (int s = 1; s < C::NKS; ++s) acc = mfma_i8(kf[s], qf[s], acc);
    }
    return acc;
  };
  auto qk = [&](int t) -> v16i {
    v4i kf[C::NKS];
    qk_load(t, kf);
    return qk_mma(kf);
  };

  // first half of the softmax of a tile (c = sq*sk*qks of the tile):
  //   (a) row max of the int32 scores and d = f16(S - rm): independent of the running max, so it
  //       shares a basic block with the PV MFMAs of the previous tile;
  //   (b) deferred running-max update (rare branch), er = exp2(rm - m), sp = f16(er / 127).
  auto sm1a = [&](const v16i& acc_in, float c, SmTile& st, int t) -> _Float16 {
    // causal tiles crossing this wave's diagonal: keys above the row's query drop out of the max
    // (INT_MIN) and get d = -inf below, so P = 0 and the tile scale sp ignores them
    const bool diag = CAUSAL && (t * C::KT + C::KT - 1 > q0);
    v16i acc = acc_in;
    if (diag) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (t * C::KT + (r & 3) + 8 * (r >> 2) + 4 * h > q0 + c32) acc[r] = INT_MIN;
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
    // S = f16(f32(acc * c)) (int8:200-203: fp32 products, then fp16); v_mul + v_cvt_pk_f16_f32 is
    // cheaper than v_fma_mix (tools/ubench) and rounds like the reference's fp32 chain
    const _Float16 rm = (_Float16)((float)mx * c);
    v2h s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      s2[j] = __builtin_bit_cast(v2h, pk_f16((float)acc[2 * j] * c, (float)acc[2 * j + 1] * c));
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
    return rm;
  };
  auto sm1b = [&](_Float16 rm, SmTile& st) {
    if (__ballot((float)rm > (float)m + C::THR) != 0) {
      const _Float16 nm = m > rm ? m : rm;
      const float r = exp2_f32((float)(_Float16)(m - nm));
      m = nm;
      l *= r;
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) o[b] *= r;
    }
    st.er = exp2_f32((float)(_Float16)(rm - m));
    st.sp = (_Float16)(st.er * (1.0f / 127.0f));
  };

  // second half: e = exp2(d), l += er * sum e, P operand (2 x 8 packed pairs = 2 x v8h)
  auto sm2 = [&](const SmTile& st, v4u* pw) {
    const v2h one2 = {(_Float16)1.0f, (_Float16)1.0f};
    v2h e[8], w[8];
    exp2_pk4(&st.d[0], &e[0]);
    exp2_pk4(&st.d[4], &e[4]);
    // row-sum of e: one packed f16 add level (pairs of values <= 1), then fp32; v_dot2c_f32_f16 is
    // avoided: beside MFMAs it issues ~5x slower than plain VALU (tools/ubench)
    float esum;   // (not 0.f + ...: a float +0 is not folded away)
    {
      const v2h p = e[0] + e[1];
      esum = (float)p[0] + (float)p[1];
    }
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      const v2h p = e[2 * j] + e[2 * j + 1];
      esum += (float)p[0] + (float)p[1];
    }
    (void)one2;
    l += esum * st.er;
    const v2h sp2 = {st.sp, st.sp};
    const _Float16 nsp = (_Float16)(-1024.0f) * st.sp;
    const v2h nsp2 = {nsp, nsp};
#ifdef QA_FWD_PTRUNC
    {
      const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
      v2h x[8], t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = e[j] * k127;
      trunc_pk4(&x[0], &t[0]);
      trunc_pk4(&x[4], &t[4]);
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j] = t[j] * sp2;
      (void)nsp2;
    }
#else
    p_operand8(e, sp2, nsp2, w);
#endif
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) pw[s][j] = __builtin_bit_cast(unsigned, w[4 * s + j]);
  };

  // O^T += Vdq^T P^T for tile t: operand loads (issued early, consumed after QK(t+1) and SM2(t))
  // and the MFMAs
  auto pv_load = [&](auto t, v8h* va) {
    const char* vl = slot_of(t);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) {
        const char* a = vl + voff[b] + 16 * s * 2 * D;
        if (AB == 6 && s == 1) { va[s * C::NDB + b] = va[b] * (_Float16)2.0f; continue; }   // half the V reads (timing)
        va[s * C::NDB + b] = __builtin_bit_cast(v8h, ds_read_tr16_x2(a, a + 8 * 2 * D));
      }
  };
  auto pv_mma = [&](const v8h* va, const v4u* pw) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) {
        if constexpr (AB == 2) {
          asm volatile("" ::"v"(va[s * C::NDB + b]), "v"(pw[s]));
        } else {
          o[b] = mfma_f16(va[s * C::NDB + b], __builtin_bit_cast(v8h, pw[s]), o[b]);
        }
      }
  };

#if defined(QA_FWD_PRIO)
  {  // co-resident workgroups (blocks b, b+256, b+512 on one CU in the first wave of dispatch) get
     // different static priorities so that their identical streams do not run in lockstep
    const int pr = (blockIdx.x >> 8) % 3;
    if (pr == 1) __builtin_amdgcn_s_setprio(1);
    else if (pr == 2) __builtin_amdgcn_s_setprio(2);
  }
#endif
#if defined(QA_FWD_SLEEP)
  {
    const int pr = (blockIdx.x >> 8) % 3;
    if (pr == 1) __builtin_amdgcn_s_sleep(QA_FWD_SLEEP);
    else if (pr == 2) { __builtin_amdgcn_s_sleep(QA_FWD_SLEEP); __builtin_amdgcn_s_sleep(QA_FWD_SLEEP); }
  }
#endif
  vmem_drain();
  __syncthreads();

  SmTile st;
  if (active) {
    const v16i acc0 = qk(0);
    if constexpr (SOFTMAX) sm1b(sm1a(acc0, cq * (float)sk_lds[0], st, 0), st);
    else st.d[0] = __builtin_bit_cast(v2h, acc0[0]);
  }
  // Steady state: one basic block per tile (except the rare running-max rescale).  The last
  // iteration computes QK / SM1 of a duplicate of the last tile (its slot holds a clamped re-load):
  // harmless (its row max cannot move m) and it keeps the loop body branch-free.
#if defined(QA_FWD_STAMP)
  unsigned long long wg_t0 = __builtin_amdgcn_s_memtime();
  // timing build: per-phase s_memtime stamps of workgroups 0..31, tiles 0..63
  unsigned long long* stamp = g_fwd_stamps + ((long)(blockIdx.x * C::WAVES + wave) * 64) * 8;
  const bool do_stamp = blockIdx.x < 32;
#define QA_STAMP(k)                                                                  \
  if (do_stamp && t < 64 && lane == 0) {                                             \
    __builtin_amdgcn_sched_barrier(0);                                               \
    stamp[t * 8 + (k)] = __builtin_amdgcn_s_memtime();                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
  }
#else
#define QA_STAMP(k)
#endif
  // one tile: SLc holds tile t, NXc tile t+1 (the slot after the last one holds a clamped duplicate),
  // DMc is the slot the DMA of tile t+3 refills
  auto step = [&](auto SLc, auto NXc, auto DMc, int t) {
    QA_STAMP(0)
    if constexpr (STREAM) {
#if defined(QA_FWD_NOBAR)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::IPW) : "memory");   // timing experiment only
#else
      ring_wait_barrier<C::IPW>();   // tile t+1 landed (t+2 may be in flight); slot (t+3)&3 is free
#endif
      QA_STAMP(1)
      dma.issue(smem_lds + slot_idx(DMc) * C::SLOT, min(t + 3, nt - 1));
    }
    if (active) {
      const int tn = min(t + 1, nt - 1);
      const float cn = cq * (float)sk_lds[tn];
      v4i kf[C::NKS];
      qk_load(NXc, kf);
      v8h va[2 * C::NDB];
#if defined(QA_FWD_VLATE)
      // the V reads join the LDS queue only after this wave's K reads have returned, so the K reads
      // of the other waves of the workgroup (all released by the same barrier) are not queued
      // behind 4 x 16 transposed V reads
      const v16i nacc = qk_mma(kf);
      __builtin_amdgcn_sched_barrier(0);
      pv_load(SLc, va);
      __builtin_amdgcn_sched_barrier(0);
#else
      pv_load(SLc, va);
#endif
#if defined(QA_FWD_SB)
      __builtin_amdgcn_sched_barrier(0);   // LDS reads issue first; the softmax VALU covers their latency
      v4u pw[2];
      sm2(st, pw);
      __builtin_amdgcn_sched_barrier(0);
      const v16i nacc = qk_mma(kf);
#elif !defined(QA_FWD_VLATE)
      const v16i nacc = qk_mma(kf);
#endif
      QA_STAMP(2)
#if !defined(QA_FWD_SB)
      v4u pw[2];
      if constexpr (SOFTMAX) {
        sm2(st, pw);
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 4; ++j) pw[s][j] = __builtin_bit_cast(unsigned, st.d[4 * s + j]) & 0x3fff3fffu;
      }
#endif
      QA_STAMP(3)
      pv_mma(va, pw);
      QA_STAMP(4)
      if constexpr (SOFTMAX) {
        const _Float16 rm = sm1a(nacc, cn, st, tn);
        QA_STAMP(5)
        sm1b(rm, st);
      } else {
        st.d[0] = __builtin_bit_cast(v2h, nacc[0]);
      }
      QA_STAMP(6)
    }
    };
#if QA_FWD_UNROLL
  static_assert(C::NSLOT == 4, "unrolled for the 4-slot ring");
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  for (int t = 0; t < nt; t += 4) {
    step(I0{}, I1{}, I3{}, t);
    if (t + 1 < nt) step(I1{}, I2{}, I0{}, t + 1);
    if (t + 2 < nt) step(I2{}, I3{}, I1{}, t + 2);
    if (t + 3 < nt) step(I3{}, I0{}, I2{}, t + 3);
  }
#else
  for (int t = 0; t < nt; ++t) step(t, t + 1, t + 3, t);
#endif
#undef QA_STAMP
  if constexpr (STREAM) vmcnt_wait_all();
  __syncthreads();   // every wave is done with the ring: its slots become the output staging area

  if (!active) return;
#if defined(QA_FWD_STAMP)
  if (tid == 0 && blockIdx.x < 8192) {   // per workgroup: start, end, HW_ID, XCC_ID
    unsigned long long* w = g_fwd_wginfo + 4L * blockIdx.x;
    w[0] = wg_t0;
    w[1] = __builtin_amdgcn_s_memtime();
    w[2] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID, 32 bits
    w[3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));   // HW_REG_XCC_ID
  }
#endif
  // ---------------- epilogue: lse = fp16(m + fp16(log2 l)); O = fp16(O / l)   (int8:252-257)
  l = pair_sum(l);
  const long qrow = head_row0 + q0 + c32;
  if (h == 0) lse[qrow] = (_Float16)((float)m + (float)(_Float16)log2_f32(l));
  static_assert(C::WAVES * RowTile<D, _Float16>::BYTES <= C::NSLOT * C::SLOT, "staging fits the ring");
  store_rows<D, _Float16>(o, 1.0f / l, smem + wave * RowTile<D, _Float16>::BYTES,
                          out + (head_row0 + q0) * D, lane);
}

template <int D, int AB, bool CAUSAL>
static int launch_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                      const void* vdq, void* out, void* lse, long bh, long sq_tok, long sk_tok, int group,
                      float qks, hipStream_t st) {
  using C = Int8FwdCfg<D>;
  const int nq = (int)((sq_tok + C::QROWS - 1) / C::QROWS);
  const int lds = C::NSLOT * C::SLOT + (int)(((sk_tok / 32) * 2 + 15) / 16 * 16);
  hipFuncSetAttribute((const void*)int8_attn_fwd_kernel<D, AB, CAUSAL>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL((int8_attn_fwd_kernel<D, AB, CAUSAL>), dim3((unsigned)(nq * bh)),
                     dim3(64 * C::WAVES), lds, st, (const int8_t*)q_i8, (const _Float16*)sq,
                     (const int8_t*)k_i8, (const _Float16*)sk, (const _Float16*)vdq, (_Float16*)out,
                     (_Float16*)lse, (int)bh, (int)sq_tok, (int)sk_tok, group, qks);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_int8_attn_fwd_ex(const void* q_i8, const void* sq, const void* k_i8,
                                      const void* sk, const void* vdq, void* out, void* lse, long bh,
                                      long sq_tok, long sk_tok, int group, int causal, int head_dim,
                                      float qks, void* stream) {
  if (sq_tok % 32 != 0 || sk_tok % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq_tok == 0) return 0;
  if (sk_tok == 0) return 1;
  hipStream_t st = (hipStream_t)stream;
#define QA_L(Dv, CV) launch_fwd<Dv, 0, CV>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, sq_tok, sk_tok, group, qks, st)
  if (head_dim == 128) return causal ? QA_L(128, true) : QA_L(128, false);
  return causal ? QA_L(64, true) : QA_L(64, false);
#undef QA_L
}

extern "C" int qattn_int8_attn_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                                   const void* vdq, void* out, void* lse, long bh, long seq,
                                   int head_dim, float qks, void* stream) {
  return qattn_int8_attn_fwd_ex(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, 0, head_dim, qks,
                                stream);
}

extern "C" int qattn_int8_attn_fwd_ablate(const void* q_i8, const void* sq, const void* k_i8,
                                          const void* sk, const void* vdq, void* out, void* lse,
                                          long bh, long seq, float qks, int ab, void* stream) {
  if (seq % 32 != 0 || bh == 0) return 1;
  hipStream_t st = (hipStream_t)stream;
  switch (ab) {
    case 1: return launch_fwd<128, 1, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
    case 2: return launch_fwd<128, 2, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
    case 3: return launch_fwd<128, 3, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
    case 4: return launch_fwd<128, 4, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
    case 5: return launch_fwd<128, 5, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
    case 6: return launch_fwd<128, 6, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
    case 7: return launch_fwd<128, 7, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
    default: return launch_fwd<128, 0, false>(q_i8, sq, k_i8, sk, vdq, out, lse, bh, seq, seq, 1, qks, st);
  }
}

#if defined(QA_FWD_STAMP)
extern "C" int qattn_fwd_stamps(void* stamps, void* wginfo) {
  hipMemcpyFromSymbol(stamps, HIP_SYMBOL(g_fwd_stamps), sizeof(g_fwd_stamps));
  hipMemcpyFromSymbol(wginfo, HIP_SYMBOL(g_fwd_wginfo), sizeof(g_fwd_wginfo));
  return 0;
}
#endif
