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
// Every bf16 rounding is the hardware RNE v_cvt_pk_bf16_f32 on pairs (unpacked with one shift /
// mask each); "#{S >= thr} > 1" is evaluated as "second-largest S of the row >= thr", with the
// row's top two values carried by v_max / v_med3 (the largest is the row max the rule needs anyway).
//
// Structure (as int8_attn_fwd.hip): 4 waves x 32 query rows per workgroup, three workgroups per CU
// (three waves per SIMD); 32-key K/V tiles stream through a 3-slot LDS ring filled by buffer
// LDS-DMA (one barrier per tile); swapped QK^T (keys in registers, one query per lane pair) so P
// feeds the PV MFMA straight from registers; V read column-wise with ds_read_b64_tr_b16.  One
// 16-key sub-tile == one k-step of the 32x32x16 PV MFMA.
//
// Causal with a V-suffix workspace (qattn_bf16_fwd_ws_ex): past a wave's diagonal tile every score
// is the fill value -126, the running max can no longer move (the diagonal tile already holds the
// fill at key == query, so m >= bf16(-126 qks)) and the beta rule cannot fire (its threshold is
// >= bf16(-126 qks) - 1e-3 > -126), so every masked sub-tile adds the same P = p to each key:
// O += p * sum_{k >= K0} V[k], l += p * (Sk - K0).  bf16_vsuffix_* compute sum_{k >= 32 b} V[k]
// once per key/value head; the tile loop stops at the workgroup's last diagonal tile and a wave
// skips the tiles past its own, replacing the masked half of the P.V MFMAs by one FMA per output.
#include <type_traits>

#include "common.h"


namespace qattn {

#ifndef QA_BF_FWD_WAVES
#define QA_BF_FWD_WAVES 4   // waves (32 queries each) per workgroup
#endif
// Occupancy (round 6): three waves per SIMD (<= 168 VGPRs; OCC), a 3-slot ring (three 4-wave
// workgroups' rings and output staging fit one CU's LDS; NSLOT), the two sub-tiles' phases one after
// the other (SEQ: A0 B0 C0 A1 B1 C1) and no QK^T one tile ahead (PIPE = 0): the third wave covers the
// latency the software pipeline and the interleaved sub-tiles covered before, in 164 instead of 188
// VGPRs at D = 128 (no spills).  Bit-identical; 2-6 % faster at configs 2 and 3, causal included
// (profiles/r06_bf16_fwd_3wave_ab.log).  The round-5 form is OCC 2, NSLOT 4, SEQ 0, PIPE 1.
#ifndef QA_BF_FWD_OCC
#define QA_BF_FWD_OCC 3
#endif
#ifndef QA_BF_FWD_NSLOT
#define QA_BF_FWD_NSLOT 3
#endif
#ifndef QA_BF_FWD_SEQ
#define QA_BF_FWD_SEQ 1
#endif
#ifndef QA_BF_FWD_PIPE
#define QA_BF_FWD_PIPE 0
#endif

template <int D>
struct Bf16FwdCfg {
  static constexpr int WAVES = QA_BF_FWD_WAVES;
  static constexpr int QROWS = 32 * WAVES;
  static constexpr int KT = 32;                 // keys per ring slot
  static constexpr int NSLOT = QA_BF_FWD_NSLOT;
  static constexpr int ROWB = 2 * D;            // bytes per K / V row
  static constexpr int NCH = ROWB / 16;         // 16-B chunks per row
  static constexpr int TILE = KT * ROWB;        // bytes per K (or V) tile
  static constexpr int SLOT = 2 * TILE;
  static constexpr int NKS = D / 16;            // f16 k-steps of QK^T
  static constexpr int NDB = D / 32;
  static constexpr int PIECES = SLOT / 1024;    // 1-KiB LDS-DMA pieces per slot
  static constexpr int IPW = PIECES / WAVES;
  static constexpr int K_SHIFT = (D == 128) ? 0 : 1;   // K swizzle = (row >> K_SHIFT) & (NCH-1)
  static constexpr int V_SHIFT = (D == 128) ? 2 : 1;   // V swizzle = (row & 3) << V_SHIFT
  // output staging passes (two halves of the columns when the ring is 3 slots: 3 workgroups per CU)
  static constexpr int STAGE_PASSES = NSLOT == 3 ? 2 : 1;
  static constexpr int STAGE_BYTES = WAVES * RowTile<D, float, STAGE_PASSES>::BYTES;
  static constexpr int LDS = (NSLOT * SLOT > STAGE_BYTES) ? NSLOT * SLOT : STAGE_BYTES;
};

template <int D>
QA_DEVICE int bk_sw(int row) {
  using C = Bf16FwdCfg<D>;
  return (row >> C::K_SHIFT) & (C::NCH - 1);
}
template <int D>
QA_DEVICE int bv_sw(int row) {
  using C = Bf16FwdCfg<D>;
  return (row & 3) << C::V_SHIFT;
}

// LDS-DMA plan of one 32-key tile: piece p < TILE/1024 is K, the rest V; lane-constant offsets.
template <int D>
struct Bf16Dma {
  using C = Bf16FwdCfg<D>;
  unsigned voff[C::IPW];
  unsigned lds_off[C::IPW];
  v4u rsrc[C::IPW];
  QA_DEVICE void init(int wave, int lane, int Sk, const void* kbase, const void* vbase) {
    constexpr int RPI = 64 / C::NCH;
    constexpr int KP = C::TILE / 1024;
#pragma unroll
    for (int i = 0; i < C::IPW; ++i) {
      const int p = wave + C::WAVES * i;
      const bool isv = p >= KP;
      const int piece = isv ? p - KP : p;
      const int row = piece * RPI + lane / C::NCH, c = lane % C::NCH;
      voff[i] = row * C::ROWB + 16 * (c ^ (isv ? bv_sw<D>(row) : bk_sw<D>(row)));
      lds_off[i] = (isv ? C::TILE : 0) + piece * 1024;
      rsrc[i] = make_rsrc(isv ? vbase : kbase, (unsigned)Sk * C::ROWB);
    }
  }
  QA_DEVICE void issue(unsigned slot_lds, int tile) const {
#pragma unroll
    for (int i = 0; i < C::IPW; ++i)
      dma16_buf(rsrc[i], voff[i], (unsigned)tile * C::TILE, slot_lds + lds_off[i]);
  }
};

// bf16 RNE of two fp32 values, returned unpacked as fp32 (and the packed pair)
QA_DEVICE unsigned rne2(float a, float b, float& ra, float& rb) {
  const unsigned w = pk_bf16(a, b);
  ra = __uint_as_float(w << 16);
  rb = __uint_as_float(w & 0xffff0000u);
  return w;
}
QA_DEVICE float rne1(float a) { return __uint_as_float(pk_bf16(a, a) & 0xffff0000u); }

// Per key/value head, per 32-key tile b: T[b][d] = sum of V[32b .. 32b+31][d] (fp32).  256
// threads: 16-B column chunks x row groups, reduced through LDS.
template <int D>
__global__ __launch_bounds__(256) void bf16_vsuffix_tiles(const __bf16* __restrict__ v,
                                                          float* __restrict__ ws, int nt) {
  constexpr int NC = D / 8, RG = 256 / NC;   // column chunks, row groups
  __shared__ float part[RG][D];
  const int bt = blockIdx.x, hkv = bt / nt, t = bt % nt;
  const int c = threadIdx.x % NC, rg = threadIdx.x / NC;
  const __bf16* src = v + ((long)hkv * nt * 32 + (long)t * 32) * D + 8 * c;
  float a[8] = {};
  for (int r = rg; r < 32; r += RG) {
    const v8bf x = *reinterpret_cast<const v8bf*>(src + (long)r * D);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] += (float)x[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[rg][8 * c + j] = a[j];
  __syncthreads();
  if (threadIdx.x < D) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < RG; ++g) s += part[g][threadIdx.x];
    ws[((long)hkv * (nt + 1) + t) * D + threadIdx.x] = s;
  }
}

// In place, per key/value head: ws[b][d] = sum_{b' >= b} T[b'][d], ws[nt][d] = 0.  1024 threads =
// NG groups of D columns; group g scans its run of tiles on top of the totals of the groups after it.
template <int D>
__global__ __launch_bounds__(1024) void bf16_vsuffix_scan(float* __restrict__ ws, int nt) {
  constexpr int NG = 1024 / D;
  __shared__ float tot[NG][D];
  const int d = threadIdx.x % D, g = threadIdx.x / D;
  const int per = (nt + NG - 1) / NG, b0 = min(g * per, nt), b1 = min(b0 + per, nt);
  float* w = ws + (long)blockIdx.x * (nt + 1) * D + d;
  float s = 0.f;
  for (int b = b0; b < b1; ++b) s += w[(long)b * D];
  tot[g][d] = s;
  __syncthreads();
  float acc = 0.f;
  for (int g2 = NG - 1; g2 > g; --g2) acc += tot[g2][d];
  for (int b = b1 - 1; b >= b0; --b) {
    acc += w[(long)b * D];
    w[(long)b * D] = acc;
  }
  if (g == 0) w[(long)nt * D] = 0.f;
}

template <int D, bool CAUSAL, bool SFX>
__global__ __launch_bounds__(64 * QA_BF_FWD_WAVES, QA_BF_FWD_OCC) void bf16_fwd_kernel(
    const _Float16* __restrict__ q, const _Float16* __restrict__ k, const __bf16* __restrict__ v,
    float* __restrict__ out, float* __restrict__ lse, int BH, int Sq, int Sk, int G, float qks,
    const float* __restrict__ vsuf) {
  static_assert(!SFX || CAUSAL, "the V-suffix path is causal only");
  using C = Bf16FwdCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nq = (Sq + C::QROWS - 1) / C::QROWS;
  int bh, qt;
  if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nq, BH, true, bh, qt);
  else xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qt * C::QROWS + wave * 32;
  const bool active = q0 < Sq;
  const int qidx = q0 + c32;                     // this lane's query row
  const float thr_eps = 0.00099945068359375f;    // bf16(1e-3): eager `bf16 - 1e-3` rounds the scalar (bf16:248)
  const int nt = Sk / C::KT;
  // SFX: the workgroup's last diagonal tile ends the loop (tiles past it are masked for every wave)
  const int nte = SFX ? min(nt, (qt * C::QROWS + C::QROWS) / C::KT) : nt;

  Bf16Dma<D> dma;
  // grouped-query attention: query head bh reads key/value head bh / G
  dma.init(wave, lane, Sk, k + (long)(bh / G) * Sk * D, v + (long)(bh / G) * Sk * D);
  const unsigned smem_lds = lds_addr(smem);
#pragma unroll
  for (int i = 0; i < C::NSLOT - 1; ++i) dma.issue(smem_lds + i * C::SLOT, min(i, nte - 1));

  v8h qf[C::NKS];
  {
    // waves past the end (ragged Sq) run on a clamped copy of the last row and store nothing, so
    // the tile loop has no per-wave branch
    const _Float16* qrow = q + ((long)bh * Sq + min(qidx, Sq - 1)) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v8h*>(qrow + 16 * s);
  }
  // lane-constant LDS offsets: K A-operand chunk (2s+h) of key row c32; V^T A-operand per d block
  int koff[C::NKS], voff[C::NDB];
#pragma unroll
  for (int s = 0; s < C::NKS; ++s) koff[s] = c32 * C::ROWB + 16 * ((2 * s + h) ^ bk_sw<D>(c32));
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int key_a = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      voff[b] = C::TILE + key_a * C::ROWB + 16 * ((d / 8) ^ bv_sw<D>(key_a)) + (d % 8) * 2;
    }
  }
  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  float m = -INFINITY;   // bf16-valued
  // l (bf16:198, initial 1 wiped by r = 0 on the first sub-tile) is accumulated by the matrix core:
  // lacc = lacc*r + ones.P, every register of lane l holding l of query l&31 (the VALU is the
  // bottleneck, the MFMA pipe has room)
  v16f lacc;
#pragma unroll
  for (int i = 0; i < 16; ++i) lacc[i] = 1.0f;
  v8bf ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;

  // ring slots are compile-time constants (the tile loop is unrolled by NSLOT) so every LDS
  // address is a lane-constant VGPR plus an instruction offset
  auto qk = [&](auto SLc) -> v16f {
    const char* kl = smem + decltype(SLc)::value * C::SLOT;
    v16f acc = v16f{};
#pragma unroll
    for (int s = 0; s < C::NKS; ++s)
      acc = mfma_f16(*reinterpret_cast<const v8h*>(kl + koff[s]), qf[s], acc);
    return acc;
  };
  // One 16-key sub-tile u of tile t (acc registers 8u .. 8u+7) in three phases, ordered per tile
  // as A0 A1 B0 B1 C0 C1 so the two sub-tiles' independent work shares one branch-free block:
  //   A: S = bf16(fp16(acc)), causal fill, the row's top two (independent of m)
  //   B: beta rule, P (bf16 pairs) and r (serial in m)
  //   C: rescale of O and l when some r != 1 (uniform branch), l += ones.P, O += P.V
  struct Sub {
    float s[8];
    float M1, M2;
    v4u pk;
    float r;
  };
  const float inf = INFINITY;
  // causal: a 16-key sub-tile whose first key is at or past the wave's last query is masked for
  // every row (S = -126 throughout, bf16:222-233): its S, top two and P need no per-score work
  auto masked = [&](int t, int u) { return CAUSAL && t * C::KT + 16 * u >= q0 + 31; };
  auto phase_a = [&](Sub& x, int t, int u, const v16f& acc) {
    if (masked(t, u)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x.s[j] = -126.0f;
      x.M1 = x.M2 = -126.0f;
      return;
    }
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const unsigned hh = pk_f16(acc[8 * u + j], acc[8 * u + j + 1]);
      const v2h p = __builtin_bit_cast(v2h, hh);
      rne2((float)p[0], (float)p[1], x.s[j], x.s[j + 1]);
    }
    const int key_t0 = t * C::KT + 16 * u;
    if (CAUSAL && key_t0 + 15 >= q0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int key = key_t0 + (j & 3) + 8 * (j >> 2) + 4 * h;
        x.s[j] = (qidx - key <= 0) ? -126.0f : x.s[j];
      }
    }
    // top two (8 here, 8 in lane l^32); fmed3(a, b, +-inf) = max / min in one instruction
    float m1 = __builtin_amdgcn_fmed3f(x.s[0], x.s[1], inf), m2 = __builtin_amdgcn_fmed3f(x.s[0], x.s[1], -inf);
#pragma unroll
    for (int j = 2; j < 8; ++j) {
      m2 = __builtin_amdgcn_fmed3f(m1, m2, x.s[j]);
      m1 = __builtin_amdgcn_fmed3f(m1, x.s[j], inf);
    }
    const auto x1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m1), __float_as_uint(m1), false, false);
    const auto x2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m2), __float_as_uint(m2), false, false);
    const float a1 = __uint_as_float(x1[0]), b1 = __uint_as_float(x1[1]);
    x.M1 = __builtin_amdgcn_fmed3f(a1, b1, inf);
    x.M2 = __builtin_amdgcn_fmed3f(   // max(min(m1, o1), m2, o2)
        __builtin_amdgcn_fmed3f(__builtin_amdgcn_fmed3f(a1, b1, -inf), __uint_as_float(x2[0]), inf),
        __uint_as_float(x2[1]), inf);
  };
  auto phase_b = [&](Sub& x, bool msk) {
    float nm = __builtin_amdgcn_fmed3f(m, rne1(x.M1 * qks), inf);   // bf16:236-239
    const float thr = rne1(nm - thr_eps);                            // bf16:248
    // #{S >= thr} > 1  <=>  second largest >= thr:  m' = 2m' (m' > 0) | 0 (m' < 0)   bf16:248-264
    const float dbl = (nm > 0.f) ? rne1(2.0f * nm) : 0.0f;
    nm = (x.M2 >= thr && nm != 0.f) ? dbl : nm;
    // P = bf16(exp2(bf16(bf16(S*qks) - nm))).  Scalar fp32 on purpose: v_pk_*_f32 issue through
    // the matrix pipe and stall ~38 cycles behind the co-resident wave's MFMAs (tools/ubench).
    if (msk) {   // every S is -126: one P for the lane's 8 scores (the same operations)
      const float p = exp2_f32(rne1(rne1(-126.0f * qks) - nm));
      const unsigned w = pk_bf16(p, p);
      x.pk = v4u{w, w, w, w};
    } else {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        float a, b;
        rne2(x.s[j] * qks, x.s[j + 1] * qks, a, b);
        rne2(a - nm, b - nm, a, b);
        x.pk[j / 2] = pk_bf16(exp2_f32(a), exp2_f32(b));
      }
    }
    x.r = rne1(exp2_f32(rne1(m - nm)));                              // bf16:276
    m = nm;
  };
  auto phase_c = [&](auto SLc, const Sub& x, int u) {
    if (__ballot(x.r != 1.0f)) {
#pragma unroll
      for (int b = 0; b < C::NDB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[b][i] = o[b][i] * x.r;
#pragma unroll
      for (int i = 0; i < 16; ++i) lacc[i] = lacc[i] * x.r;
    }
    const v8bf pb8 = __builtin_bit_cast(v8bf, x.pk);
    lacc = mfma_bf16(ones, pb8, lacc);                               // l = l*r + sum P   (bf16:279)
    const char* vl = smem + decltype(SLc)::value * C::SLOT;
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const char* a = vl + voff[b] + 16 * u * C::ROWB;
      const v8bf va = __builtin_bit_cast(v8bf, ds_read_tr16_x2(a, a + 8 * C::ROWB));
      o[b] = mfma_bf16(va, pb8, o[b]);                               // bf16:285
    }
  };

  vmem_drain();
  __syncthreads();
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  v16f acc = v16f{};
  if (QA_BF_FWD_PIPE) acc = qk(I0{});
  // tile t lives in slot t % NSLOT; at tile t the slot (t+1) % NSLOT holds tile min(t+1, nt-1)
  auto step = [&](auto SLc, auto NXc, auto FRc, int t) {
    // tile t+1 landed (later tiles may be in flight); slot (t + NSLOT - 1) % NSLOT is free
    ring_wait_barrier<(C::NSLOT - 3) * C::IPW>();
    dma.issue(smem_lds + decltype(FRc)::value * C::SLOT, min(t + C::NSLOT - 1, nte - 1));
    if (!(SFX && masked(t, 0))) {   // SFX: a tile past the wave's diagonal is in the suffix
      // (a tile masked for the whole wave needs no S: its QK^T MFMAs are skipped)
      v16f nacc = v16f{};
      if (QA_BF_FWD_PIPE) {
        if (!masked(t + 1, 0)) nacc = qk(NXc);
      } else if (!masked(t, 0)) {
        acc = qk(SLc);
      }
      if (QA_BF_FWD_SEQ) {
        {
          Sub x0;
          phase_a(x0, t, 0, acc);
          phase_b(x0, masked(t, 0));
          phase_c(SLc, x0, 0);
        }
        Sub x1;
        phase_a(x1, t, 1, acc);
        phase_b(x1, masked(t, 1));
        phase_c(SLc, x1, 1);
      } else {
        Sub x0, x1;
        phase_a(x0, t, 0, acc);
        phase_a(x1, t, 1, acc);
        phase_b(x0, masked(t, 0));
        phase_b(x1, masked(t, 1));
        phase_c(SLc, x0, 0);
        phase_c(SLc, x1, 1);
      }
      if (QA_BF_FWD_PIPE) acc = nacc;
    }
  };
  if constexpr (C::NSLOT == 4) {
    for (int t = 0; t < nte; t += 4) {
      step(I0{}, I1{}, I3{}, t);
      if (t + 1 < nte) step(I1{}, I2{}, I0{}, t + 1);
      if (t + 2 < nte) step(I2{}, I3{}, I1{}, t + 2);
      if (t + 3 < nte) step(I3{}, I0{}, I2{}, t + 3);
    }
  } else {
    static_assert(C::NSLOT == 3, "ring of 3 or 4 slots");
    for (int t = 0; t < nte; t += 3) {
      step(I0{}, I1{}, I2{}, t);
      if (t + 1 < nte) step(I1{}, I2{}, I0{}, t + 1);
      if (t + 2 < nte) step(I2{}, I0{}, I1{}, t + 2);
    }
  }
  if constexpr (SFX) {
    // the masked keys K0 .. Sk-1 of this wave, all at once (see the header)
    const int K0 = q0 + 32;
    if (K0 < Sk) {
      const float cfill = rne1(-126.0f * qks);
      const float nm = __builtin_amdgcn_fmed3f(m, cfill, inf);   // == m (kept for the general rule)
      const float r = rne1(exp2_f32(rne1(m - nm)));
      if (__ballot(r != 1.0f)) {
#pragma unroll
        for (int b = 0; b < C::NDB; ++b)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[b][i] = o[b][i] * r;
#pragma unroll
        for (int i = 0; i < 16; ++i) lacc[i] = lacc[i] * r;
      }
      m = nm;
      const float p = rne1(exp2_f32(rne1(cfill - m)));
      const float* vs = vsuf + ((long)(bh / G) * (nt + 1) + K0 / C::KT) * D + 4 * h;
#pragma unroll
      for (int b = 0; b < C::NDB; ++b)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const v4f x = *reinterpret_cast<const v4f*>(vs + 32 * b + 8 * g);
#pragma unroll
          for (int j = 0; j < 4; ++j) o[b][4 * g + j] += p * x[j];
        }
      lacc[0] += p * (float)(Sk - K0);
    }
  }
  vmcnt_wait_all();
  __syncthreads();   // the ring becomes the output staging area
  if (!active) return;
  const long row0 = (long)bh * Sq + q0;
  const float l = lacc[0];
  if (h == 0) lse[row0 + c32] = m + log2_f32(l);                 // bf16:288
  store_rows<D, float, C::STAGE_PASSES>(o, 1.0f / l, smem + wave * RowTile<D, float, C::STAGE_PASSES>::BYTES,
                                        out + row0 * D, lane);
}

}  // namespace qattn

using namespace qattn;

extern "C" long qattn_bf16_fwd_ws_bytes(long bh_kv, long sk, int head_dim) {
  return bh_kv * (sk / 32 + 1) * head_dim * 4;
}

extern "C" int qattn_bf16_fwd_ws_ex(const void* q, const void* k, const void* v, void* out, void* lse,
                                    long bh, long sq, long sk, int group, int causal, int head_dim,
                                    float qks, void* ws, void* stream) {
  if (sq % 32 != 0 || sk % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq == 0) return 0;
  if (ws != nullptr && (reinterpret_cast<uintptr_t>(ws) & 15) != 0) return 1;
  hipStream_t st = (hipStream_t)stream;
  const int nt = (int)(sk / 32);
  const bool sfx = causal && ws != nullptr && nt > 0;
  if (sfx) {   // the per-head V suffix sums the causal loop stops short of
    const long hkv = bh / group;
    if (head_dim == 128) {
      hipLaunchKernelGGL(bf16_vsuffix_tiles<128>, dim3((unsigned)(hkv * nt)), dim3(256), 0, st, (const __bf16*)v, (float*)ws, nt);
      hipLaunchKernelGGL(bf16_vsuffix_scan<128>, dim3((unsigned)hkv), dim3(1024), 0, st, (float*)ws, nt);
    } else {
      hipLaunchKernelGGL(bf16_vsuffix_tiles<64>, dim3((unsigned)(hkv * nt)), dim3(256), 0, st, (const __bf16*)v, (float*)ws, nt);
      hipLaunchKernelGGL(bf16_vsuffix_scan<64>, dim3((unsigned)hkv), dim3(1024), 0, st, (float*)ws, nt);
    }
  }
#define QA_LAUNCH(Dv, CV, SV)                                                                    \
  {                                                                                              \
    using C = Bf16FwdCfg<Dv>;                                                                    \
    const int nq = (int)((sq + C::QROWS - 1) / C::QROWS);                                        \
    { static LdsGrant granted_; lds_grant((const void*)bf16_fwd_kernel<Dv, CV, SV>, C::LDS, granted_); } \
    hipLaunchKernelGGL((bf16_fwd_kernel<Dv, CV, SV>), dim3((unsigned)(nq * bh)), dim3(64 * C::WAVES), \
                       C::LDS, st, (const _Float16*)q, (const _Float16*)k, (const __bf16*)v,     \
                       (float*)out, (float*)lse, (int)bh, (int)sq, (int)sk, group, qks,          \
                       (const float*)ws);                                                        \
  }
  if (head_dim == 128) {
    if (sfx) QA_LAUNCH(128, true, true) else if (causal) QA_LAUNCH(128, true, false) else QA_LAUNCH(128, false, false)
  } else {
    if (sfx) QA_LAUNCH(64, true, true) else if (causal) QA_LAUNCH(64, true, false) else QA_LAUNCH(64, false, false)
  }
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_bf16_fwd_ex(const void* q, const void* k, const void* v, void* out, void* lse,
                                 long bh, long sq, long sk, int group, int causal, int head_dim,
                                 float qks, void* stream) {
  return qattn_bf16_fwd_ws_ex(q, k, v, out, lse, bh, sq, sk, group, causal, head_dim, qks, nullptr, stream);
}

extern "C" int qattn_bf16_fwd(const void* q, const void* k, const void* v, void* out, void* lse, long bh,
                              long sq, long sk, int head_dim, int causal, float qks, void* stream) {
  return qattn_bf16_fwd_ex(q, k, v, out, lse, bh, sq, sk, 1, causal, head_dim, qks, stream);
}
