// FlashAttention-2 backward (algorithm 4) for gfx950; replaces helion_flash_atten_2_algo_4_bwd
// (attention_bf16.py:299-448) with the build-contract fixes of SURVEY F3:
//   P  = exp2(qks * q.k - lse)      (causal: strictly-lower kept, else qks*S := -128)  bf16:376-392
//   dV = P^T dO                                                                          bf16:399
//   dP = dO V^T ;  D = rowsum(dO * O) (once per row, prep kernel)                        bf16:405,416
//   dS = P * (dP - D)                (reference: S * (dP - D), F3)                       bf16:421
//   dQ = sm_scale * dS K ;  dK = sm_scale * dS^T Q   (reference: qk_scale, racy dq RMW)   bf16:427-441
//
// Deterministic by construction: each output row block has one owner workgroup that accumulates it
// in registers over all tiles of the other side (S and dP are recomputed per kernel; no atomics, no
// read-modify-write of global memory).
//
// MFMA precisions: S = Q K^T in fp16 (inputs are fp16, products exact, fp32 accumulate);
// dP, dV, dK, dQ in bf16 (dO, dS rounded to bf16; Q/K rounded to bf16 for the dK/dQ products;
// V is bf16 already), fp32 accumulate.  Causal tiles that are entirely masked contribute
// exp2(-128 - lse) < 2^-120 per element and are skipped.
#include <type_traits>

#include "common.h"

namespace qattn {

// ------------------------------------------------------------------------------------------ prep
// One pass over dO (fp32) and O: dO_bf = bf16(dO) (the dP / dV operand image) and
// LD[row] = {lse[row], D = rowsum(dO * O)} (bf16:416, once per row instead of per tile), interleaved
// so one 256-B LDS-DMA per 32-row tile brings both.  16 lanes per row, 8 floats per lane (D=128).
template <int D>
__global__ __launch_bounds__(256) void bf16_bwd_prep_kernel(const float* __restrict__ dO,
                                                            const float* __restrict__ O,
                                                            const float* __restrict__ lse,
                                                            __bf16* __restrict__ dO_bf,
                                                            float2* __restrict__ LD, long rows) {
  constexpr int LPR = D / 8;  // lanes per row
  const long row = ((long)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = (threadIdx.x % LPR) * 8;
  float acc = 0.f;
  if (row < rows) {
    const v4f* a = reinterpret_cast<const v4f*>(dO + row * D + c);
    const v4f* b = reinterpret_cast<const v4f*>(O + row * D + c);
    const v4f a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
    acc = a0[0] * b0[0] + a0[1] * b0[1] + a0[2] * b0[2] + a0[3] * b0[3] +
          a1[0] * b1[0] + a1[1] * b1[1] + a1[2] * b1[2] + a1[3] * b1[3];
    v4u pk = {pk_bf16(a0[0], a0[1]), pk_bf16(a0[2], a0[3]), pk_bf16(a1[0], a1[1]), pk_bf16(a1[2], a1[3])};
    *reinterpret_cast<v4u*>(dO_bf + row * D + c) = pk;
  }
#pragma unroll
  for (int o = LPR / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if (row < rows && (threadIdx.x % LPR) == 0) LD[row] = float2{lse[row], acc};
}

// y = bf16(x) (RNE) for fp16 x: the transposed-read images of q (dK product) and k (dQ product)
__global__ __launch_bounds__(256) void f16_to_bf16_kernel(const _Float16* __restrict__ x,
                                                          __bf16* __restrict__ y, long n8) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const v8h a = reinterpret_cast<const v8h*>(x)[i];
  v4u w;
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = pk_bf16((float)a[2 * j], (float)a[2 * j + 1]);
  reinterpret_cast<v4u*>(y)[i] = w;
}

// ------------------------------------------------------------- dV, dK, dQ: one kernel template
// A wave owns 32 rows of one side X whose fragments stay in registers (B operands) and streams
// 32-row tiles of the other side Y through an LDS ring filled by buffer LDS-DMA:
//   ROLE_DV: X = K (fp16)           Y = {Q fp16 rows, dO bf16 tr image, LD}   S -> P -> dV += dO^T P
//   ROLE_DK: X = K (fp16), V (bf16) Y = {Q fp16 rows, dO bf16 rows, Q bf16 tr image, LD}
//                                                                           S, dP -> dS -> dK += Q^T dS
//   ROLE_DQ: X = Q (fp16), dO (bf16) Y = {K fp16 rows, V bf16 rows, K bf16 tr image}
//                                                                           S, dP -> dS -> dQ += K^T dS^T
// S = Q K^T on the fp16 MFMA (exact products, fp32 accumulation), dP on the bf16 MFMA (dO, V bf16),
// P = exp2(S*qks - lse) and dS = P*(dP - D) in fp32, then bf16 operands of the accumulating bf16
// MFMA against the transposed (ds_read_b64_tr_b16) image of the third operand.  Software pipelined by
// one tile: the products of tile t+1 are issued before the accumulation of tile t, and the fp32
// P / dS of tile t+1 are computed beside its MFMAs.
//   ROLE_DKV (bf16_bwd_dkv_kernel below, the default path): X = K, V; Y = {Q fp16 rows, dO bf16
//             rows, Q bf16 tr image, dO bf16 tr image, LD}; S and P computed once for dV and dK.
// The split DV + DK kernels (S recomputed in each) remain as qattn_bf16_bwd_split_ex.
enum B16Role { B16_DV = 0, B16_DK = 1, B16_DQ = 2, B16_DKV = 3 };
#ifndef QA_B16_DV_OCC
#define QA_B16_DV_OCC 2
#endif
#ifndef QA_B16_DMA_P
#define QA_B16_DMA_P 1   // fused dK+dV: only the P waves issue the ring DMA (dS waves never wait on vmcnt)
#endif
#ifndef QA_B16_DQ_WAVES
#define QA_B16_DQ_WAVES 8   // dQ workgroup: 4 or 8 waves of 32 queries (8 halves the k/v stream per query)
#endif
#ifndef QA_B16_DV_NSLOT
#define QA_B16_DV_NSLOT 3
#endif

template <int D, int ROLE>
struct B16Cfg {
  static constexpr int ROWB = 2 * D;
  static constexpr int NCH = ROWB / 16;
  static constexpr int T16 = 32 * ROWB;                     // one 32-row 16-bit tile
  static constexpr bool TWO = ROLE != B16_DV;               // S and dP
  static constexpr bool HAS_LD = ROLE != B16_DQ;            // {lse, D} per row of the streamed side
  static constexpr bool FUSED = ROLE == B16_DKV;
  // FUSED at D=128: one dO image serves both the row reads (dP) and the tr reads (dV), under the
  // swizzle b16_csw that is conflict-free for both; D=64 keeps a separate dO tr image
  static constexpr bool MERGE = FUSED && D == 128;
  static constexpr int NREG = FUSED ? (MERGE ? 3 : 4) : TWO ? 3 : 2;   // 16-bit regions per slot
  static constexpr int NROW = FUSED ? 2 : NREG - 1;         // row-read regions come first
  static constexpr int YA = 0, YB = T16, TR = NROW * T16, TR2 = MERGE ? YB : 3 * T16, LDO = NREG * T16;
  static constexpr int SLOT = NREG * T16 + (HAS_LD ? 256 : 0);
  static constexpr int NSLOT = (ROLE == B16_DV) ? QA_B16_DV_NSLOT : 3;
  static constexpr int WAVES = FUSED ? 8 : (ROLE == B16_DQ && D == 128) ? QA_B16_DQ_WAVES : 4;
  static constexpr int XROWS = 32 * (FUSED ? 4 : WAVES);    // own rows per workgroup
  static constexpr int NP = T16 / 1024;                     // 1-KiB LDS-DMA pieces per region
  static constexpr int INST = NREG * NP;
  static constexpr int DMA_WAVES = (FUSED && QA_B16_DMA_P) ? 4 : WAVES;   // waves issuing the DMA
  static constexpr int IPW16 = INST / DMA_WAVES;
  static constexpr int IPW = IPW16 + (HAS_LD ? 1 : 0);      // VMEM ops per wave per tile
  static constexpr int NKS = D / 16;
  static constexpr int NDB = D / 32;
  static constexpr int STAGE = WAVES * RowTile<D, float, 2>::BYTES;   // epilogue in two column halves
  static constexpr int PBUF = NSLOT * SLOT;                 // FUSED: fp32 P hand-over, 2 tiles
  static constexpr int PB_WAVE = 32 * 32 * 4, PB_TILE = 4 * PB_WAVE;
  static constexpr int RING = PBUF + (FUSED ? 2 * PB_TILE : 0);
  static constexpr int LDS = (RING > STAGE) ? RING : STAGE;
  static_assert(INST % DMA_WAVES == 0, "DMA pieces split evenly over the waves");
};
template <int D>
QA_DEVICE int b16_rsw(int row) { return (D == 128) ? (row & 15) : ((row >> 1) & 7); }   // row reads
template <int D>
QA_DEVICE int b16_tsw(int row) { return (row & 3) << ((D == 128) ? 2 : 1); }            // tr reads
// both (D = 128): ds_read_b128 row reads see 16 distinct chunks per 16-lane group, and
// ds_read_b64_tr_b16 reads of 4 rows x 4 chunks per 32-lane group see 16 distinct chunks; unlike
// b16_tsw it is not invariant under row += 8, so tr reads keep one offset per 8-row half
QA_DEVICE int b16_csw(int row) { return (row & 15) ^ ((row & 3) << 2); }

template <int D, int ROLE>
struct B16Dma {
  using G = B16Cfg<D, ROLE>;
  unsigned voff[G::IPW16];
  unsigned lds_off[G::IPW16];
  v4u rsrc[G::IPW16];
  v4u ld_rsrc;
  bool ld_on;
  // region r of a slot is filled from src[r] (row-swizzled for r < NROW, tr-swizzled after; the
  // merged dO region with b16_csw)
  QA_DEVICE void init(int wave, int lane, int Sy, const char* const* src, const char* ld) {
    constexpr int RPI = 64 / G::NCH;
#pragma unroll
    for (int i = 0; i < G::IPW16; ++i) {
      const int p = wave % G::DMA_WAVES + G::DMA_WAVES * i;
      const int r = p / G::NP, q = p % G::NP;
      const bool is_tr = r >= G::NROW;
      const int row = q * RPI + lane / G::NCH, c = lane % G::NCH;
      const int sw = (G::MERGE && r == 1) ? b16_csw(row) : is_tr ? b16_tsw<D>(row) : b16_rsw<D>(row);
      voff[i] = row * G::ROWB + 16 * (c ^ sw);
      lds_off[i] = r * G::T16 + q * 1024;
      rsrc[i] = make_rsrc(src[r], (unsigned)Sy * G::ROWB);
    }
    if constexpr (G::HAS_LD) ld_rsrc = make_rsrc(ld, (unsigned)Sy * 8);
    ld_on = !G::FUSED || wave == G::DMA_WAVES - 1;   // FUSED: one wave brings the {lse, D} rows
    dma_on = wave < G::DMA_WAVES;
  }
  bool dma_on;
  QA_DEVICE void issue(unsigned slot_lds, int t, int lane) const {
    if (!dma_on) return;
#pragma unroll
    for (int i = 0; i < G::IPW16; ++i)
      dma16_buf(rsrc[i], voff[i], (unsigned)t * G::T16, slot_lds + lds_off[i]);
    if constexpr (G::HAS_LD)
      if (ld_on) dma4_buf(ld_rsrc, 4 * lane, (unsigned)t * 256, slot_lds + G::LDO);
  }
};

template <int D, int ROLE, bool CAUSAL>
__global__ __launch_bounds__((64 * B16Cfg<D, ROLE>::WAVES), ROLE == B16_DV ? QA_B16_DV_OCC : 2) void
bf16_bwd_kernel(const _Float16* __restrict__ xa, const __bf16* __restrict__ xb,
                const _Float16* __restrict__ ya, const __bf16* __restrict__ yb,
                const __bf16* __restrict__ ytr, const __bf16* __restrict__ ytr2,
                const float2* __restrict__ yld, const float2* __restrict__ xld, float* __restrict__ out,
                float* __restrict__ out2, int BH, int Sx, int Ny, int ydiv, int Smod, float qks,
                float osc, float osc2, __bf16* __restrict__ /*ws: fused kernel only*/) {
  using G = B16Cfg<D, ROLE>;
  constexpr bool TWO = G::TWO;
  static_assert(!G::FUSED, "B16_DKV runs bf16_bwd_dkv_kernel");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nxb = (Sx + G::XROWS - 1) / G::XROWS;
  int bh, xt;
  if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nxb, BH, ROLE == B16_DQ, bh, xt);
  else xcd_remap(blockIdx.x, nxb, BH, bh, xt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int x0 = xt * G::XROWS + wave * 32;
  const bool active = x0 < Sx;
  const int xi = x0 + c32;                      // this lane's own row
  // own head bh streams the Ny rows from (bh / ydiv) * Ny: dV/dK the G query heads of a key/value
  // head (contiguous, Ny = G * Sq), dQ the key/value head of a query head (ydiv = G, Ny = Sk);
  // positions of streamed rows are taken mod Smod
  const long hx = (long)bh * Sx, hy = (long)(bh / ydiv) * Ny;
  // tile range: causal tiles masked for the whole workgroup are skipped (they contribute
  // exp2(-128 - lse) < 2^-120 per element)
  int t0 = 0, t1 = Ny / 32;
  if (CAUSAL) {
    if (ROLE == B16_DQ) t1 = min(t1, (xt * G::XROWS + G::XROWS) / 32);   // keys >= every query
    else if (Ny == Smod) t0 = min(t1, (xt * G::XROWS) / 32);              // queries <= every key
  }
  const int nt = t1 - t0;
  // causal dQ accumulates, per wave, the key tiles of its 128-query block (floor(kt/4) <=
  // floor(qt/4)) whatever the workgroup size: the same tiles as the dK+dV kernel's records cover
  const int t1w = (CAUSAL && ROLE == B16_DQ) ? min(t1, (x0 / 128) * 4 + 4) : t1;

  B16Dma<D, ROLE> dma;
  {
    const char* ysrc[4] = {reinterpret_cast<const char*>(ya + hy * D),
                           reinterpret_cast<const char*>((TWO ? yb : ytr) + hy * D),
                           reinterpret_cast<const char*>(ytr + hy * D),
                           reinterpret_cast<const char*>(ytr + hy * D)};
    dma.init(wave, lane, Ny, ysrc, reinterpret_cast<const char*>(yld + hy));
  }
  const unsigned smem_lds = lds_addr(smem);
  if (nt > 0) {
#pragma unroll
    for (int i = 0; i < G::NSLOT - 1; ++i) dma.issue(smem_lds + i * G::SLOT, t0 + min(i, nt - 1), lane);
  }

  // own fragments (B operands): lane holds X[xi][16s + 8h .. +8]
  const int xr = min(xi, Sx - 1);
  v8h xfa[G::NKS];
  v8bf xfb[TWO ? G::NKS : 1];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) {
    xfa[s] = *reinterpret_cast<const v8h*>(xa + (hx + xr) * D + 16 * s + 8 * h);
    if constexpr (TWO) xfb[s] = *reinterpret_cast<const v8bf*>(xb + (hx + xr) * D + 16 * s + 8 * h);
  }
  float lsex = 0.f, Dx = 0.f;
  if constexpr (!G::HAS_LD) {
    const float2 v = xld[hx + xr];
    lsex = v.x;
    Dx = v.y;
  }
  // lane-constant LDS offsets: row-read A operand chunk (2s+h) of row c32; tr A operand per d block
  int roff[G::NKS], troff[G::NDB];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s) roff[s] = c32 * G::ROWB + 16 * ((2 * s + h) ^ b16_rsw<D>(c32));
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int row = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < G::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      troff[b] = G::TR + row * G::ROWB + 16 * ((d / 8) ^ b16_tsw<D>(row)) + (d % 8) * 2;
    }
  }
  v16f acc[G::NDB];
#pragma unroll
  for (int b = 0; b < G::NDB; ++b) acc[b] = v16f{};

  // tile t lives in ring slot (t - t0) % NSLOT; the loop is unrolled by NSLOT so the slot is a
  // compile-time constant and every LDS address a lane-constant VGPR plus an instruction offset
  auto slot = [&](auto SLc) -> const char* { return smem + decltype(SLc)::value * G::SLOT; };
  // S (fp16 MFMA) and dP (bf16 MFMA) of the tile in slot SL, rows = streamed side, lane = own row
  auto products = [&](auto SLc, v16f& sa, v16f& pa) {
    const char* base = slot(SLc);
    sa = v16f{};
    pa = v16f{};
#pragma unroll
    for (int s = 0; s < G::NKS; ++s) {
      sa = mfma_f16(*reinterpret_cast<const v8h*>(base + G::YA + roff[s]), xfa[s], sa);
      if constexpr (TWO) pa = mfma_bf16(*reinterpret_cast<const v8bf*>(base + G::YB + roff[s]), xfb[s], pa);
    }
  };
  // fp32 P (DV) or dS (DK, DQ) of tile t
  auto values = [&](auto SLc, int t, const v16f& sa, const v16f& pa, float* X) {
    const int y0 = (32 * t) % Smod;
    const bool mask = CAUSAL && (ROLE == B16_DQ ? (y0 + 31 >= x0) : (y0 <= x0 + 31));
    if constexpr (G::HAS_LD) {
      const float* ld = reinterpret_cast<const float*>(slot(SLc) + G::LDO);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f a = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h));
        const v4f b = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h) + 4);
        const float lse_r[4] = {a[0], a[2], b[0], b[2]};
        const float d_r[4] = {a[1], a[3], b[1], b[3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g + j;
          float sc = sa[i] * qks;                                          // bf16:376-377
          if (mask && y0 + 8 * g + 4 * h + j - xi <= 0) sc = -128.0f;       // bf16:379-389
          const float p = exp2_f32(sc - lse_r[j]);                         // bf16:392
          if constexpr (ROLE == B16_DV) X[i] = p;
          else X[i] = p * (pa[i] - d_r[j]);                                // dS = P (dP - D), F3
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float sc = sa[i] * qks;
        if (mask && xi - (y0 + (i & 3) + 8 * (i >> 2) + 4 * h) <= 0) sc = -128.0f;
        X[i] = exp2_f32(sc - lsex) * (pa[i] - Dx);
      }
    }
  };
  auto operand = [&](const float* X, v8bf* op) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      v4u w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = pk_bf16(X[8 * s + 2 * j], X[8 * s + 2 * j + 1]);
      op[s] = __builtin_bit_cast(v8bf, w);
    }
  };
  auto tr_load = [&](auto SLc, v8bf* ta) {
    const char* base = slot(SLc);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < G::NDB; ++b) {
        const char* a = base + troff[b] + 16 * s * G::ROWB;
        ta[s * G::NDB + b] = __builtin_bit_cast(v8bf, ds_read_tr16_x2(a, a + 8 * G::ROWB));
      }
  };

  vmem_drain();
  __syncthreads();
  static_assert(G::NSLOT == 3, "the tile loop below is unrolled for a 3-slot ring");
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  float X[16];
  // one tile: slot SL holds tile t, slot NX = (SL+1)%3 tile min(t+1, t1-1) (the DMA clamps to the
  // last tile, so the slot after the last one holds a duplicate and the loop body stays uniform)
  auto step = [&](auto SLc, auto NXc, int t) {
    ring_wait_barrier<(G::NSLOT - 3) * G::IPW>();   // tile t+1 landed; the slot of tile t-1 is free
    dma.issue(smem_lds + ((decltype(SLc)::value + G::NSLOT - 1) % G::NSLOT) * G::SLOT,
              min(t + G::NSLOT - 1, t1 - 1), lane);
    const int tn = min(t + 1, t1 - 1);
    v8bf ta[2 * G::NDB];
    tr_load(SLc, ta);
    v16f sa, pa;
    products(NXc, sa, pa);
    v8bf op[2];
    operand(X, op);
    if (t < t1w) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int b = 0; b < G::NDB; ++b) acc[b] = mfma_bf16(ta[s * G::NDB + b], op[s], acc[b]);
    }
    values(NXc, tn, sa, pa, X);
  };
  if (nt > 0) {
    {
      v16f sa, pa;
      products(I0{}, sa, pa);
      values(I0{}, t0, sa, pa, X);
    }
    for (int t = t0; t < t1; t += 3) {
      step(I0{}, I1{}, t);
      if (t + 1 < t1) step(I1{}, I2{}, t + 1);
      if (t + 2 < t1) step(I2{}, I0{}, t + 2);
    }
  }
  vmcnt_wait_all();
  __syncthreads();   // the ring becomes the output staging area
  if (!active) return;
  store_rows<D, float, 2>(acc, osc, smem + wave * RowTile<D, float, 2>::BYTES, out + (hx + x0) * D, lane);
}

// ---------------------------------------------------------------- fused dK + dV, paired waves
// One workgroup owns 128 keys of one key/value head; every 32 keys have two waves on one SIMD:
//   P wave  (waves 0-3, K fp16 fragments):  S -> P = exp2(S*qks - lse) -> dV += dO^T P
//   dS wave (waves 4-7, V bf16 fragments):  dP -> dS = P (dP - D)     -> dK += Q^T dS
// The P wave hands its fp32 P of tile t+1 to the dS wave through LDS (two tile buffers); the dS
// wave uses it one step later, after the ring barrier, so it runs one tile behind.  Both waves
// carry 16 MFMAs per tile (S or dP, then dV or dK), S and P are computed once, and the P / dS
// operands and accumulation order are those of the DV / DK kernels: dK, dV are bit-identical to
// the split path.  Registers: one fragment set + one accumulator per wave, two waves per SIMD.
// WS: the dS wave also stores each bf16 dS tile (exactly its dK operand) as a 2 KiB record, row-
// major [key][query], at ((query head * Sq/32 + query tile) * Sk/32 + key tile) * 2 KiB, for
// bf16_bwd_dqw_kernel.
template <int D, bool CAUSAL, bool WS>
__global__ __launch_bounds__(512, 2) void bf16_bwd_dkv_kernel(
    const _Float16* __restrict__ xa, const __bf16* __restrict__ xb, const _Float16* __restrict__ ya,
    const __bf16* __restrict__ yb, const __bf16* __restrict__ ytr, const __bf16* __restrict__ ytr2,
    const float2* __restrict__ yld, const float2* __restrict__ xld, float* __restrict__ out,
    float* __restrict__ out2, int BH, int Sx, int Ny, int ydiv, int Smod, float qks, float osc,
    float osc2, __bf16* __restrict__ ws) {
  using G = B16Cfg<D, B16_DKV>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nxb = (Sx + G::XROWS - 1) / G::XROWS;
  int bh, xt;
  if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nxb, BH, false, bh, xt);
  else xcd_remap(blockIdx.x, nxb, BH, bh, xt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool pwave = wave < 4;
  const int kw = wave & 3;
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int x0 = xt * G::XROWS + kw * 32;
  const bool active = x0 < Sx;
  const int xi = x0 + c32;
  const long hx = (long)bh * Sx, hy = (long)(bh / ydiv) * Ny;
  int t0 = 0, t1 = Ny / 32;
  if (CAUSAL && Ny == Smod) t0 = min(t1, (xt * G::XROWS) / 32);   // queries <= every key
  const int nt = t1 - t0;

  B16Dma<D, B16_DKV> dma;
  {
    const char* ysrc[4] = {reinterpret_cast<const char*>(ya + hy * D),
                           reinterpret_cast<const char*>(yb + hy * D),
                           reinterpret_cast<const char*>(ytr + hy * D),
                           reinterpret_cast<const char*>(ytr2 + hy * D)};
    dma.init(wave, lane, Ny, ysrc, reinterpret_cast<const char*>(yld + hy));
  }
  const unsigned smem_lds = lds_addr(smem);
  if (nt > 0) {
#pragma unroll
    for (int i = 0; i < G::NSLOT - 1; ++i) dma.issue(smem_lds + i * G::SLOT, t0 + min(i, nt - 1), lane);
  }
  const int xr = min(xi, Sx - 1);
  // row reads: P wave Q (region YA), dS wave dO (YB); tr reads: P wave dO (TR2), dS wave Q (TR).
  // troff[s][half][b]: rows 16 s + 8 half + 4 h + i16/4 of the tr read
  const bool csw_rows = G::MERGE && !pwave, csw_tr = G::MERGE && pwave;
  int roff[G::NKS], troff[2][2][G::NDB];
#pragma unroll
  for (int s = 0; s < G::NKS; ++s)
    roff[s] = c32 * G::ROWB + 16 * ((2 * s + h) ^ (csw_rows ? b16_csw(c32) : b16_rsw<D>(c32)));
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int treg = pwave ? G::TR2 : G::TR;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int row = 16 * s + 8 * hf + 4 * h + (i16 >> 2);
        const int sw = csw_tr ? b16_csw(row) : b16_tsw<D>(row);
#pragma unroll
        for (int b = 0; b < G::NDB; ++b) {
          const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
          troff[s][hf][b] = treg + row * G::ROWB + 16 * ((d / 8) ^ sw) + (d % 8) * 2;
        }
      }
  }
  v16f acc[G::NDB];
#pragma unroll
  for (int b = 0; b < G::NDB; ++b) acc[b] = v16f{};
  // P hand-over: tile t's P of key wave kw at PBUF + ((t - t0) & 1) * PB_TILE + kw * PB_WAVE, lane-
  // interleaved v4f (conflict-free b128 accesses)
  auto pbuf = [&](int t) { return reinterpret_cast<v4f*>(smem + G::PBUF + ((t - t0) & 1) * G::PB_TILE +
                                                         kw * G::PB_WAVE) + lane; };
  auto slot = [&](auto SLc) -> const char* { return smem + decltype(SLc)::value * G::SLOT; };
  auto operand = [&](const float* X, v8bf* op) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      v4u w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = pk_bf16(X[8 * s + 2 * j], X[8 * s + 2 * j + 1]);
      op[s] = __builtin_bit_cast(v8bf, w);
    }
  };
  auto accumulate = [&](auto SLc, const v8bf* op) {
    const char* base = slot(SLc);
    v8bf ta[2 * G::NDB];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < G::NDB; ++b)
        ta[s * G::NDB + b] =
            __builtin_bit_cast(v8bf, ds_read_tr16_x2(base + troff[s][0][b], base + troff[s][1][b]));
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < G::NDB; ++b) acc[b] = mfma_bf16(ta[s * G::NDB + b], op[s], acc[b]);
  };
  static_assert(G::NSLOT == 3, "the tile loops below are unrolled for a 3-slot ring");
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  float X[16];
  // an active dS wave of the WS kernel ends each step with its record stores, younger than the
  // DMA of tile t+1: they may stay in flight across the barrier
  const bool st_wave = WS && !pwave && active;
  auto ring = [&](auto SLc, int t) {
    static_assert(G::NSLOT == 3, "vmcnt counts below assume a 3-slot ring");
    if (G::DMA_WAVES == 4 && !pwave) {
      // no ring DMA in this wave: its record stores stay in flight
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else if (st_wave) ring_wait_barrier<2>();            // tile t+1 landed, P(t) written; slot t-1 free
    else ring_wait_barrier<0>();
    dma.issue(smem_lds + ((decltype(SLc)::value + G::NSLOT - 1) % G::NSLOT) * G::SLOT,
              min(t + G::NSLOT - 1, t1 - 1), lane);
  };
  vmem_drain();
  __syncthreads();
  if (pwave) {
    v8h xf[G::NKS];
#pragma unroll
    for (int s = 0; s < G::NKS; ++s)
      xf[s] = *reinterpret_cast<const v8h*>(xa + (hx + xr) * D + 16 * s + 8 * h);
    auto sprod = [&](auto SLc) {
      const char* base = slot(SLc);
      v16f sa{};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) sa = mfma_f16(*reinterpret_cast<const v8h*>(base + G::YA + roff[s]), xf[s], sa);
      return sa;
    };
    // P of tile t in X (as the DV kernel) and in hand-over buffer pb
    auto pvals = [&](auto SLc, int t, const v16f& sa, v4f* pb) {
      const int y0 = (32 * t) % Smod;
      const bool mask = CAUSAL && (y0 <= x0 + 31);
      const float* ld = reinterpret_cast<const float*>(slot(SLc) + G::LDO);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f a = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h));
        const v4f b = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h) + 4);
        const float lse_r[4] = {a[0], a[2], b[0], b[2]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g + j;
          float sc = sa[i] * qks;                                          // bf16:376-377
          if (mask && y0 + 8 * g + 4 * h + j - xi <= 0) sc = -128.0f;       // bf16:379-389
          X[i] = exp2_f32(sc - lse_r[j]);                                  // bf16:392
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) pb[64 * g] = v4f{X[4 * g], X[4 * g + 1], X[4 * g + 2], X[4 * g + 3]};
    };
    // branch-free: at the last tile P(t1-1) is recomputed into the buffer of tile t+1, whose
    // previous content P(t-1) the dS wave consumed before this step's barrier
    auto step = [&](auto SLc, auto NXc, int t) {
      ring(SLc, t);
      const v16f sa = sprod(NXc);
      v8bf op[2];
      operand(X, op);
      accumulate(SLc, op);                   // dV += dO^T P(t)
      pvals(NXc, min(t + 1, t1 - 1), sa, pbuf(t + 1));
    };
    if (nt > 0) {
      pvals(I0{}, t0, sprod(I0{}), pbuf(t0));
      for (int t = t0; t < t1; t += 3) {
        step(I0{}, I1{}, t);
        if (t + 1 < t1) step(I1{}, I2{}, t + 1);
        if (t + 2 < t1) step(I2{}, I0{}, t + 2);
      }
    }
  } else {
    v8bf xf[G::NKS];
#pragma unroll
    for (int s = 0; s < G::NKS; ++s)
      xf[s] = *reinterpret_cast<const v8bf*>(xb + (hx + xr) * D + 16 * s + 8 * h);
    auto dprod = [&](auto SLc) {
      const char* base = slot(SLc);
      v16f pa{};
#pragma unroll
      for (int s = 0; s < G::NKS; ++s) pa = mfma_bf16(*reinterpret_cast<const v8bf*>(base + G::YB + roff[s]), xf[s], pa);
      return pa;
    };
    v16f pa = v16f{};
    auto step = [&](auto SLc, auto NXc, int t) {
      ring(SLc, t);
      const v4f* pb = pbuf(t);
      v4f pv[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) pv[g] = pb[64 * g];
      const v16f pn = dprod(NXc);
      // dS(t) = P(t) (dP(t) - D), as the DK kernel (F3)
      const float* ld = reinterpret_cast<const float*>(slot(SLc) + G::LDO);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f a = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h));
        const v4f b = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h) + 4);
        const float d_r[4] = {a[1], a[3], b[1], b[3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) X[4 * g + j] = pv[g][j] * (pa[4 * g + j] - d_r[j]);
      }
      v8bf op[2];
      operand(X, op);
      accumulate(SLc, op);                   // dK += Q^T dS(t)
      pa = pn;
      if constexpr (WS) {
        // lane (key c32, half h) holds queries 8g + 4h + j of X[4g + j] (op[g/2], words 2(g%2)..+1)
        if (active) {
          char* r = reinterpret_cast<char*>(ws) +
                    (((long)bh * (Ny / 32) + t) * (Sx / 32) + x0 / 32) * 2048 + c32 * 64;
          // one permlane32_swap per word pair: the h=0 lane gets queries 0-15 of its key row, the
          // h=1 lane queries 16-31; each writes 32 contiguous bytes (two b128 stores)
          const v4u w0 = __builtin_bit_cast(v4u, op[0]), w1 = __builtin_bit_cast(v4u, op[1]);
          v4u lo, hi;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const auto x = __builtin_amdgcn_permlane32_swap(w0[i], w1[i], false, false);
            lo[i] = x[0];
            hi[i] = x[1];
          }
          *reinterpret_cast<v4u*>(r + 32 * h) = v4u{lo[0], lo[1], hi[0], hi[1]};
          *reinterpret_cast<v4u*>(r + 32 * h + 16) = v4u{lo[2], lo[3], hi[2], hi[3]};
        }
      }
    };
    if (nt > 0) {
      pa = dprod(I0{});
      for (int t = t0; t < t1; t += 3) {
        step(I0{}, I1{}, t);
        if (t + 1 < t1) step(I1{}, I2{}, t + 1);
        if (t + 2 < t1) step(I2{}, I0{}, t + 2);
      }
    }
  }
  vmcnt_wait_all();
  __syncthreads();   // the ring becomes the output staging area
  if (!active) return;
  store_rows<D, float, 2>(acc, pwave ? osc2 : osc, smem + wave * RowTile<D, float, 2>::BYTES,
                          (pwave ? out2 : out) + (hx + x0) * D, lane);
}

// ------------------------------------------------------------------- dQ from the dS records
// dQ = sms * dS K without recomputing S, dP: 8 waves x 32 queries stream the bf16 k image (L2-
// resident, 4-slot ring) and their own 2 KiB dS records (HBM, 5-slot ring, non-temporal).  A
// record [key][query] read with ds_read_b64_tr_b16 is the dQ MFMA's B operand in the key order of
// the k image read, i.e. exactly the operand the recomputing DQ kernel builds from its registers:
// dq is bit-identical to it.  Causal: each wave visits the key tiles the recomputing kernel's
// 128-query workgroup visits (floor(kt/4) <= floor(qt/4)), which are the tiles the fused dK+dV
// kernel writes.
template <int D>
struct B16DqwCfg {
  static constexpr int WAVES = 8;
  static constexpr int ROWB = 2 * D;
  static constexpr int T16 = 32 * ROWB;
  static constexpr int NSLOT = 4, RSLOT = 5;
  static constexpr int REC = WAVES * 2048;
  static constexpr int RBASE = NSLOT * T16;
  static constexpr int NP16 = T16 / 1024;
  static constexpr int IPK = (NP16 + WAVES - 1) / WAVES;
  static constexpr int NDB = D / 32;
  static constexpr int RING = RBASE + RSLOT * REC;
  static constexpr int STAGE = WAVES * RowTile<D, float, 2>::BYTES;
  static constexpr int LDS = RING > STAGE ? RING : STAGE;
};

template <int D, bool CAUSAL>
__global__ __launch_bounds__(512, 2) void bf16_bwd_dqw_kernel(const __bf16* __restrict__ ws,
                                                              const __bf16* __restrict__ kbf,
                                                              float* __restrict__ dq, int BH, int Sq,
                                                              int Sk, int G, float sms) {
  using W = B16DqwCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (Sq + 32 * W::WAVES - 1) / (32 * W::WAVES);
  int bh, qb;
  if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nqb, BH, true, bh, qb);
  else xcd_remap(blockIdx.x, nqb, BH, bh, qb);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qb * 32 * W::WAVES + wave * 32;
  const bool active = q0 < Sq;
  const int nqt = Sq / 32, nkt = Sk / 32;
  const long kv_row0 = (long)(bh / G) * Sk;
  const int nt = CAUSAL ? min(nkt, 8 * qb + 8) : nkt;                      // workgroup's tiles
  const int ntw = CAUSAL ? min(nkt, (q0 / 128) * 4 + 4) : nkt;             // this wave's tiles
  const long rec0 = ((long)bh * nqt + (active ? q0 / 32 : 0)) * nkt;

  unsigned kvoff[W::IPK], klds[W::IPK];
  v4u krsrc[W::IPK];
#pragma unroll
  for (int i = 0; i < W::IPK; ++i) {
    int pc = wave + W::WAVES * i;
    if (pc >= W::NP16) pc = wave % W::NP16;
    constexpr int NCH = W::ROWB / 16, RPI = 64 / NCH;
    const int row = pc * RPI + lane / NCH, c = lane % NCH;
    kvoff[i] = row * W::ROWB + 16 * (c ^ b16_tsw<D>(row));
    klds[i] = pc * 1024;
    krsrc[i] = make_rsrc(kbf + kv_row0 * D, (unsigned)Sk * W::ROWB);
  }
  const v4u rrsrc = make_rsrc(ws + rec0 * 1024, active ? (unsigned)nkt * 2048u : 0u);
  const unsigned smem_lds = lds_addr(smem);
  auto issue_k = [&](int t) {
    const unsigned sl = smem_lds + (t % W::NSLOT) * W::T16;
#pragma unroll
    for (int i = 0; i < W::IPK; ++i)
      dma16_buf(krsrc[i], kvoff[i], (unsigned)min(t, nt - 1) * W::T16, sl + klds[i]);
  };
  auto issue_r = [&](int t) {   // each record is read once: non-temporal
    const unsigned sl = smem_lds + W::RBASE + (t % W::RSLOT) * W::REC + wave * 2048;
    const unsigned so = (unsigned)min(t, nt - 1) * 2048u;
    dma16_buf_nt(rrsrc, 16u * lane, so, sl);
    dma16_buf_nt(rrsrc, 16u * lane, so + 1024u, sl + 1024u);
  };
  if (nt > 0) {
#pragma unroll
    for (int i = 0; i < W::NSLOT - 1; ++i) issue_k(i);
    for (int i = 0; i < W::RSLOT - 1; ++i) issue_r(i);
  }
  int troff[W::NDB];
  int rtro;
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int row = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < W::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      troff[b] = row * W::ROWB + 16 * ((d / 8) ^ b16_tsw<D>(row)) + (d % 8) * 2;
    }
    rtro = row * 64 + 2 * (16 * gg + 4 * (i16 & 3));
  }
  v16f acc[W::NDB];
#pragma unroll
  for (int b = 0; b < W::NDB; ++b) acc[b] = v16f{};

  vmem_drain();
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    // tile t's k image landed (and its record, issued earlier): younger than the k DMA of tile t
    // are the 2 record DMAs issued with it and the k + record DMAs of the two iterations since
    ring_wait_barrier<2 + (W::NSLOT - 2) * (W::IPK + 2)>();
    issue_k(t + W::NSLOT - 1);
    issue_r(t + W::RSLOT - 1);
    if (active && t < ntw) {
      const char* kb = smem + (t % W::NSLOT) * W::T16;
      const char* rb = smem + W::RBASE + (t % W::RSLOT) * W::REC + wave * 2048 + rtro;
      v8bf ta[2 * W::NDB], op[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int b = 0; b < W::NDB; ++b) {
          const char* a = kb + troff[b] + 16 * s * W::ROWB;
          ta[s * W::NDB + b] = __builtin_bit_cast(v8bf, ds_read_tr16_x2(a, a + 8 * W::ROWB));
        }
        op[s] = __builtin_bit_cast(v8bf, ds_read_tr16_x2(rb + 16 * s * 64, rb + 16 * s * 64 + 8 * 64));
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int b = 0; b < W::NDB; ++b) acc[b] = mfma_bf16(ta[s * W::NDB + b], op[s], acc[b]);
    }
  }
  vmcnt_wait_all();
  __syncthreads();   // the rings become the output staging area
  if (!active) return;
  store_rows<D, float, 2>(acc, sms, smem + wave * RowTile<D, float, 2>::BYTES,
                          dq + ((long)bh * Sq + q0) * D, lane);
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_bf16_bwd_prep(const void* dO, const void* O, const void* lse, void* dO_bf,
                                   void* LD, long bh, long seq, int head_dim, void* stream) {
  if (head_dim != 64 && head_dim != 128) return 1;
  const long rows = bh * seq;
  if (rows == 0) return 0;
  const int rpb = 256 / (head_dim / 8);
  dim3 grid((unsigned)((rows + rpb - 1) / rpb)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL((bf16_bwd_prep_kernel<128>), grid, block, 0, st, (const float*)dO,
                       (const float*)O, (const float*)lse, (__bf16*)dO_bf, (float2*)LD, rows);
  else
    hipLaunchKernelGGL((bf16_bwd_prep_kernel<64>), grid, block, 0, st, (const float*)dO,
                       (const float*)O, (const float*)lse, (__bf16*)dO_bf, (float2*)LD, rows);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_f16_to_bf16(const void* x, void* y, long n, void* stream) {
  if (n % 8 != 0) return 1;
  const long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(f16_to_bf16_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const _Float16*)x, (__bf16*)y, n8);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

struct B16Out {
  void* out;
  void* out2;
  float osc, osc2;
};
template <int D, int ROLE, bool CAUSAL, bool WS>
static void launch_b16c(const void* xa, const void* xb, const void* ya, const void* yb, const void* ytr,
                        const void* ytr2, const void* yld, const void* xld, B16Out o, long bh, long sx,
                        long ny, int ydiv, long smod, float qks, void* ws, hipStream_t st) {
  using G = B16Cfg<D, ROLE>;
  auto kern = [] {
    if constexpr (ROLE == B16_DKV) return bf16_bwd_dkv_kernel<D, CAUSAL, WS>;
    else return bf16_bwd_kernel<D, ROLE, CAUSAL>;
  }();
  { static LdsGrant granted_; lds_grant((const void*)kern, G::LDS, granted_); }
  const int nb = (int)((sx + G::XROWS - 1) / G::XROWS);
  hipLaunchKernelGGL(kern, dim3((unsigned)(nb * bh)), dim3(64 * G::WAVES),
                     G::LDS, st, (const _Float16*)xa, (const __bf16*)xb, (const _Float16*)ya,
                     (const __bf16*)yb, (const __bf16*)ytr, (const __bf16*)ytr2, (const float2*)yld,
                     (const float2*)xld, (float*)o.out, (float*)o.out2, (int)bh, (int)sx, (int)ny,
                     ydiv, (int)smod, qks, o.osc, o.osc2, (__bf16*)ws);
}
template <int D, int ROLE>
static void launch_b16(const void* xa, const void* xb, const void* ya, const void* yb, const void* ytr,
                       const void* ytr2, const void* yld, const void* xld, B16Out o, long bh, long sx,
                       long ny, int ydiv, long smod, int causal, float qks, hipStream_t st,
                       void* ws = nullptr) {
#define QA_L(C, W) launch_b16c<D, ROLE, C, W>(xa, xb, ya, yb, ytr, ytr2, yld, xld, o, bh, sx, ny, ydiv, \
                                              smod, qks, ws, st)
  if (ROLE == B16_DKV && ws) {
    if (causal) QA_L(true, true); else QA_L(false, true);
  } else {
    if (causal) QA_L(true, false); else QA_L(false, false);
  }
#undef QA_L
}
template <int D, bool CAUSAL>
static void launch_dqw_b16c(const void* ws, const void* k_bf, void* dq, long bh, long sq, long sk,
                            int group, float sms, hipStream_t st) {
  using W = B16DqwCfg<D>;
  { static LdsGrant granted_; lds_grant((const void*)bf16_bwd_dqw_kernel<D, CAUSAL>, W::LDS, granted_); }
  const int nb = (int)((sq + 32 * W::WAVES - 1) / (32 * W::WAVES));
  hipLaunchKernelGGL((bf16_bwd_dqw_kernel<D, CAUSAL>), dim3((unsigned)(nb * bh)), dim3(64 * W::WAVES),
                     W::LDS, st, (const __bf16*)ws, (const __bf16*)k_bf, (float*)dq, (int)bh, (int)sq,
                     (int)sk, group, sms);
}

// bh = batch * query heads; key/value tensors have bh / group heads of sk rows
template <int D>
static void bf16_bwd_d(const void* q, const void* k, const void* v, const void* dO_bf, const void* LD,
                       const void* q_bf, const void* k_bf, void* dq, void* dk, void* dv, long bh,
                       long sq, long sk, int group, int causal, float qks, float sms, bool split,
                       void* ws, hipStream_t st) {
  const long bkv = bh / group, ny = group * sq;
  if (ws) {
    // dK + dV storing the dS records, then dQ from the records
    launch_b16<D, B16_DKV>(k, v, q, dO_bf, q_bf, dO_bf, LD, nullptr, {dk, dv, sms, 1.0f}, bkv, sk, ny, 1,
                           sq, causal, qks, st, ws);
    if (causal) launch_dqw_b16c<D, true>(ws, k_bf, dq, bh, sq, sk, group, sms, st);
    else launch_dqw_b16c<D, false>(ws, k_bf, dq, bh, sq, sk, group, sms, st);
    return;
  }
  if (split) {
    // dV: own K / streamed Q rows, dO tr image, LD
    launch_b16<D, B16_DV>(k, nullptr, q, nullptr, dO_bf, nullptr, LD, nullptr, {dv, nullptr, 1.0f, 0.f},
                          bkv, sk, ny, 1, sq, causal, qks, st);
    // dK: own K, V / streamed Q rows, dO rows, Q bf16 tr image, LD
    launch_b16<D, B16_DK>(k, v, q, dO_bf, q_bf, nullptr, LD, nullptr, {dk, nullptr, sms, 0.f}, bkv, sk,
                          ny, 1, sq, causal, qks, st);
  } else {
    // dK + dV: own K, V / streamed Q rows, dO rows, Q bf16 tr image, dO bf16 tr image, LD
    launch_b16<D, B16_DKV>(k, v, q, dO_bf, q_bf, dO_bf, LD, nullptr, {dk, dv, sms, 1.0f}, bkv, sk, ny, 1,
                           sq, causal, qks, st);
  }
  // dQ: own Q, dO (+ LD of their rows) / streamed K rows, V rows, K bf16 tr image
  launch_b16<D, B16_DQ>(q, dO_bf, k, v, k_bf, nullptr, nullptr, LD, {dq, nullptr, sms, 0.f}, bh, sq, sk,
                        group, sk, causal, qks, st);
}

static int bf16_bwd_entry(const void* q, const void* k, const void* v, const void* dO_bf,
                          const void* LD, const void* q_bf, const void* k_bf, void* dq, void* dk,
                          void* dv, long bh, long sq, long sk, int group, int causal, int head_dim,
                          float qks, float sms, bool split, void* ws, void* stream) {
  if (sq % 32 != 0 || sk % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sq == 0 || sk == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    bf16_bwd_d<128>(q, k, v, dO_bf, LD, q_bf, k_bf, dq, dk, dv, bh, sq, sk, group, causal, qks, sms,
                    split, ws, st);
  else
    bf16_bwd_d<64>(q, k, v, dO_bf, LD, q_bf, k_bf, dq, dk, dv, bh, sq, sk, group, causal, qks, sms,
                   split, ws, st);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_bf16_bwd_ex(const void* q, const void* k, const void* v, const void* dO_bf,
                                 const void* LD, const void* q_bf, const void* k_bf, void* dq, void* dk,
                                 void* dv, long bh, long sq, long sk, int group, int causal,
                                 int head_dim, float qks, float sms, void* stream) {
  return bf16_bwd_entry(q, k, v, dO_bf, LD, q_bf, k_bf, dq, dk, dv, bh, sq, sk, group, causal, head_dim,
                        qks, sms, false, nullptr, stream);
}

// bytes of the dS record workspace of qattn_bf16_bwd_ws_ex (-1 on invalid sizes)
extern "C" long qattn_bf16_bwd_ws_bytes(long bh, long sq, long sk) {
  if (bh < 0 || sq < 0 || sk < 0 || sq % 32 != 0 || sk % 32 != 0) return -1;
  return bh * (sq / 32) * (sk / 32) * 2048;
}

extern "C" int qattn_bf16_bwd_ws_ex(const void* q, const void* k, const void* v, const void* dO_bf,
                                    const void* LD, const void* q_bf, const void* k_bf, void* dq, void* dk,
                                    void* dv, long bh, long sq, long sk, int group, int causal,
                                    int head_dim, float qks, float sms, void* ws, void* stream) {
  if (!ws) return 1;
  return bf16_bwd_entry(q, k, v, dO_bf, LD, q_bf, k_bf, dq, dk, dv, bh, sq, sk, group, causal, head_dim,
                        qks, sms, false, ws, stream);
}

extern "C" int qattn_bf16_bwd_split_ex(const void* q, const void* k, const void* v, const void* dO_bf,
                                       const void* LD, const void* q_bf, const void* k_bf, void* dq,
                                       void* dk, void* dv, long bh, long sq, long sk, int group,
                                       int causal, int head_dim, float qks, float sms, void* stream) {
  return bf16_bwd_entry(q, k, v, dO_bf, LD, q_bf, k_bf, dq, dk, dv, bh, sq, sk, group, causal, head_dim,
                        qks, sms, true, nullptr, stream);
}

extern "C" int qattn_bf16_bwd(const void* q, const void* k, const void* v, const void* dO_bf,
                              const void* LD, const void* q_bf, const void* k_bf, void* dq, void* dk,
                              void* dv, long bh, long sq, long sk, int head_dim, int causal, float qks,
                              float sms, void* stream) {
  return qattn_bf16_bwd_ex(q, k, v, dO_bf, LD, q_bf, k_bf, dq, dk, dv, bh, sq, sk, 1, causal, head_dim,
                           qks, sms, stream);
}
