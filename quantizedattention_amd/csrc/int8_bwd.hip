// SageAttention-3 8-bit attention backward for gfx950; replaces helion_atten_int8_hl_dot_bwd
// (attention_int8.py:264-432) with the build-contract fixes of SURVEY F4, keeping the reference's
// quantisation recipe (per 32x32 (q-tile, k-tile) pair, Bq = Bkv = 32):
//   S    = (i32(q_i8 . k_i8) * sq) * sk * qks                          int8:352-355
//   P    = exp2(S - lse)                                                int8:360
//   sP   = max(P) / 127 over the tile;  P_i8 = trunc(P / sP)           int8:363-365
//   dV  += (P_i8^T . dO_i8) * s_dO * sP                                 int8:375-378 (F4: accumulate)
//   dP   = i32(dO_i8 . v_i8) * s_dO * sv ;  D = fp16(rowsum(fp16(dO*O))) int8:382-398
//   dS   = P * (dP - D)                       (reference: S * (dP - D), F4)   int8:399
//   s_dS = max|dS| / 127 over the tile;  dS_i8 = trunc(dS / s_dS)     int8:403-405
//   dQ  += (dS_i8 . k_i8) * s_dS * sk * sm_scale  (reference: qk_scale, racy fp16 RMW, k_mean term)
//   dK  += (dS_i8^T . q_i8) * s_dS * sq * sm_scale (reference: overwrite per q-tile)
// S and P stay in fp32 here (the reference rounds S and S - lse to fp16; the difference is far below
// the int8 quantisation step and is covered by the oracle tolerance, tests/test_gpu_int8.py).
//
// MFMA use: S and dP (scales uniform per 32x32 tile; feed elementwise work) on
// v_mfma_i32_32x32x32_i8.  The three accumulating products fold their per-tile scalar into the
// quantised operand -- bf16(P_i8 * sP * s_dO), bf16(dS_i8 * s_dS * sq|sk) -- and multiply exact
// integer-valued bf16 copies of dO_i8 / q_i8 / k_i8 on v_mfma_f32_32x32x16_bf16 with fp32
// accumulation: the same sums up to one bf16 rounding of the scaled operand, without a per-tile
// i32->f32 dequantisation of D-wide accumulators.
//
// Kernel A (dK, dV): workgroup = 4 waves x 32 keys; streams 32-row query tiles (int8 row images of
// q and dO for S / dP, bf16 transposed images for dK / dV, {lse, D} per row) through a 3-stage LDS
// ring filled by LDS-DMA two tiles ahead; one barrier per tile.  Query rows in registers, key on
// the lane.  Kernel B (dQ): workgroup = 4 waves x 32 queries; streams 32-key tiles (int8 k, v row
// images, bf16 transposed k image) the same way; keys in registers, query on the lane.  Both compute
// each (q-tile, k-tile) dS tile with the same operation order, so tile scales and dS_i8 agree bit
// for bit.  Tile-wide maxima use DPP + permlane reductions.  No atomics: deterministic.
#include <climits>
#include <type_traits>
#include <cstdlib>

#include "common.h"

namespace qattn {

template <int D>
struct I8BwdCfg {
  static constexpr int NKS8 = D / 32;    // i8 k-steps over D
  static constexpr int NDB = D / 32;     // 32-wide d blocks of the accumulators
  static constexpr int T8 = 32 * D;      // 32-row int8 tile bytes
  static constexpr int T16 = 64 * D;     // 32-row bf16 tile bytes
};
// LDS image swizzles: int8 rows (read by rows for the int8 MFMAs) and bf16 tr images (read by
// ds_read_b64_tr_b16 for the bf16 MFMAs); conflict-free for both access patterns.
template <int D>
QA_DEVICE int i8_sw(int row) { return (row >> ((D == 128) ? 1 : 2)) & (D / 16 - 1); }
template <int D>
QA_DEVICE int t16_sw(int row) { return (row & 3) << ((D == 128) ? 2 : 1); }

// Quantise 16 values with the tile scale and emit the bf16 operand  trunc(x / s) * c.
QA_DEVICE void quant_operand(const float* x, float inv, float c, v8bf* out) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    v4u w;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i0 = 8 * s + 2 * j;
      w[j] = pk_bf16(__builtin_truncf(x[i0] * inv) * c, __builtin_truncf(x[i0 + 1] * inv) * c);
    }
    out[s] = __builtin_bit_cast(v8bf, w);
  }
}

// ------------------------------------------------------------------------------------ prep
// QA_PREP_HOIST: all loads of a block before its arithmetic (bit-identical; bwd_prep 100 -> 93-95 us
// at config 3, tools/ab_quant.py); 0 = the per-row-group order hipcc serialises on the LD stores
#ifndef QA_PREP_HOIST
#define QA_PREP_HOIST 1
#endif
// One wave per 32-row block of dO (and O), one pass over both:
//   sdO = f16(amax|dO| / 127), dO_i8 = trunc(f16(dO / sdO))      (int8:372-374, same quantiser)
//   img = bf16(dO_i8)  (exact; the dV product's transposed-read image; optional)
//   LD[row] = {f32(lse[row]), f32(f16(sum_d f32(f16(dO*O))))}    (int8:360, int8:398)
template <int D, bool IMG>
__global__ __launch_bounds__(256) void int8_bwd_prep_kernel(
    const _Float16* __restrict__ dO, const _Float16* __restrict__ O, const _Float16* __restrict__ lse,
    int8_t* __restrict__ idx, _Float16* __restrict__ scale, __bf16* __restrict__ img,
    float2* __restrict__ LD, long nblocks) {
  constexpr int ELEMS = 32 * D;
  constexpr int ITERS = ELEMS / 512;   // 8 halfs per lane per iteration
  constexpr int TPR = D / 8;           // lanes per row
  const int lane = threadIdx.x & 63;
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblocks) return;
  const _Float16* xb = dO + blk * ELEMS;
  const _Float16* ob = O + blk * ELEMS;
  v8h v[ITERS];
  float amax = 0.f;
#if QA_PREP_HOIST
  // every load of the block first (dO, O and the lse of the lane's row group), then the arithmetic:
  // one HBM round trip per wave instead of one per row group (hipcc otherwise keeps each group's
  // loads behind the previous group's LD store)
  v8h ov[ITERS];
  _Float16 lsev[ITERS];
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int e = (i * 64 + lane) * 8;
    v[i] = *reinterpret_cast<const v8h*>(xb + e);
    ov[i] = *reinterpret_cast<const v8h*>(ob + e);
    lsev[i] = lse[blk * 32 + e / D];
  }
#endif
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int e = (i * 64 + lane) * 8;
#if QA_PREP_HOIST
    const v8h o = ov[i];
#else
    v[i] = *reinterpret_cast<const v8h*>(xb + e);
    const v8h o = *reinterpret_cast<const v8h*>(ob + e);
#endif
    float dsum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      amax = fmaxf(amax, fabsf((float)v[i][j]));
      dsum += (float)(_Float16)((float)v[i][j] * (float)o[j]);
    }
#pragma unroll
    for (int m = TPR / 2; m >= 1; m >>= 1) dsum += __shfl_xor(dsum, m);
    if (lane % TPR == 0) {
      const long row = blk * 32 + e / D;
#if QA_PREP_HOIST
      LD[row] = float2{(float)lsev[i], (float)(_Float16)dsum};
#else
      LD[row] = float2{(float)lse[row], (float)(_Float16)dsum};
#endif
    }
  }
  amax = wave_max_f(amax);
  const _Float16 s16 = (_Float16)(amax / 127.0f);
  const float s = (float)s16;
  const float r = quant_rcp(s);
  if (lane == 0) scale[blk] = s16;
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int e = (i * 64 + lane) * 8;
    unsigned lo, hi;
    float qf[8];
    quant8(v[i], s, r, lo, hi, qf);   // (common.h: the reference's division, exactly)
    *reinterpret_cast<v2u*>(idx + blk * ELEMS + e) = v2u{lo, hi};
    if constexpr (IMG) {
      const v4u w = {pk_bf16(qf[0], qf[1]), pk_bf16(qf[2], qf[3]), pk_bf16(qf[4], qf[5]),
                     pk_bf16(qf[6], qf[7])};
      *reinterpret_cast<v4u*>(img + blk * ELEMS + e) = w;
    }
  }
}
// y = bf16(x) for int8 x (exact): 16 bytes in, 32 bytes out per thread
__global__ __launch_bounds__(256) void i8_to_bf16_kernel(const int8_t* __restrict__ x,
                                                         __bf16* __restrict__ y, long n16) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n16) return;
  const v4i w = reinterpret_cast<const v4i*>(x)[i];
  v4u lo, hi;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    unsigned p[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float a = (float)((w[k] << (24 - 16 * j)) >> 24);
      const float b = (float)((w[k] << (16 - 16 * j)) >> 24);
      p[j] = (__float_as_uint(a) >> 16) | (__float_as_uint(b) & 0xffff0000u);
    }
    if (k < 2) { lo[2 * k] = p[0]; lo[2 * k + 1] = p[1]; }
    else { hi[2 * k - 4] = p[0]; hi[2 * k - 3] = p[1]; }
  }
  reinterpret_cast<v4u*>(y)[2 * i] = lo;
  reinterpret_cast<v4u*>(y)[2 * i + 1] = hi;
}

// ------------------------------------------------------------ dV, dK, dQ: one kernel template
// Every backward product has the same shape.  A wave owns 32 rows of one side X (keys for dV/dK,
// queries for dQ) whose int8 fragments stay in registers, and streams 32-row tiles of the other
// side Y through a 4-slot LDS ring (buffer LDS-DMA, lane-constant swizzled source offsets):
//   ROLE_DV:  X = K     Y = {Q8, dO image, LD}                S     -> P      -> dV += dO^T P
//   ROLE_DK:  X = K, V  Y = {Q8, dO8, q image, LD}            S, dP -> dS     -> dK += q^T dS
//   ROLE_DKV: X = K, V  Y = {Q8, dO8, q image, dO image, LD}  S, dP -> P, dS  -> dK and dV
//   ROLE_DQ:  X = Q, dO Y = {K8, V8, k image}                 S, dP -> dS     -> dQ += k^T dS^T
// S and dP are int8 MFMAs (32x32x32) on the quantised operands; P = exp2(S*c1 - lse) and
// dS = P*(dP*c2 - D) in fp32 (c1 = sq*(sk*qks), c2 = sdO*sv, identical in all kernels so the
// per-tile quantisation of P and dS is the same everywhere); P / dS are quantised per 32x32 tile
// (amax/127, trunc, int8:363-365, 403-405) and enter a bf16 32x32x16 MFMA as the exact bf16 value
// trunc(x/s) * s * s_other, against the exact bf16 image of the other int8 operand.
// PIPE: software pipeline by one tile (the int8 MFMAs of tile t+1 are issued before the
// quantisation of tile t, the fp32 P/dS of tile t+1 are computed beside the bf16 MFMAs of tile t);
// ROLE_DKV (two fp32 accumulators) runs unpipelined with 8 waves per workgroup instead.
enum BwdRole { ROLE_DV = 0, ROLE_DK = 1, ROLE_DQ = 2, ROLE_DKV = 3 };
#ifndef QA_DKV_PIPE
#define QA_DKV_PIPE 0
#endif
// Stagger (MI355X_MICROARCH.md "Two waves per SIMD", item 9): the second half of the fused dK+dV
// workgroup (the second wave on every SIMD) runs the pipelined order, half a tile out of phase with
// its partner, so the two waves of a SIMD are not in the same phase (MFMA vs VALU) at the same time.
// Measured 1.5-5 % faster than both waves unpipelined (tools/ab_bwd.py, four boxes).
#ifndef QA_DKV_STAGGER
#define QA_DKV_STAGGER 1
#endif
#ifndef QA_DKV_I8DV_COST
#define QA_DKV_I8DV_COST 0
#endif
// fused dK+dV workgroup shape (A/B builds): waves (32 keys each) and LDS ring slots
#ifndef QA_DKV_WAVES
#define QA_DKV_WAVES 8
#endif
#ifndef QA_DKV_NSLOT
#define QA_DKV_NSLOT 4
#endif
// cache policy of the dS record stores (builtin aux: 2 = nt, 16 = sc1)
// QA_DKV_HG: causal fused dK+dV grid order -- longest-first within groups of this many heads
// per XCD (0: longest-first over all heads, xcd_remap_lpt)
#ifndef QA_DKV_HG
#define QA_DKV_HG 4
#endif
#ifndef QA_DQW_HG   // (the same for the causal dQ-from-records grid)
#define QA_DQW_HG 0
#endif
#ifndef QA_DKV_PRIO
#define QA_DKV_PRIO 0
#endif
#ifndef QA_DQW_PRIO
#define QA_DQW_PRIO 0
#endif
#ifndef QA_BWD_PACK_ASM
#define QA_BWD_PACK_ASM 1
#endif


template <int D, int ROLE>
struct BwdCfg {
  using C = I8BwdCfg<D>;
  static constexpr bool TWO = ROLE != ROLE_DV;              // S and dP (else S only)
  static constexpr bool HAS_LD = ROLE != ROLE_DQ;           // per-row {lse, D} of the streamed side
  static constexpr bool WANT_P = ROLE == ROLE_DV || ROLE == ROLE_DKV;
  static constexpr bool WANT_DS = ROLE != ROLE_DV;
  static constexpr int NTR = (ROLE == ROLE_DKV) ? 2 : 1;    // transposed images per tile
  static constexpr int WAVES = (ROLE == ROLE_DKV) ? QA_DKV_WAVES : 4;
  static constexpr bool PIPE = ROLE != ROLE_DKV;
  static constexpr int Y8A = 0;
  static constexpr int Y8B = C::T8;
  static constexpr int TR = TWO ? 2 * C::T8 : C::T8;        // image of the dS product (or P for DV)
  static constexpr int TR2 = TR + C::T16;                   // DKV: dO image (P product)
  static constexpr int LDO = TR + NTR * C::T16;
  static constexpr int SLOT = LDO + (HAS_LD ? 256 : 0);
  static constexpr int NSLOT = (ROLE == ROLE_DKV) ? QA_DKV_NSLOT : 4;
  static constexpr int NP8 = C::T8 / 1024, NP16 = C::T16 / 1024;
  static constexpr int INST = NP8 * (TWO ? 2 : 1) + NTR * NP16;   // 1-KiB pieces per tile
  static constexpr int IPW16 = (INST + WAVES - 1) / WAVES;
  // every wave also loads the tile's 256-B LD block (duplicate writes of the same bytes): one
  // uniform instruction instead of a per-wave branch
  static constexpr int IPW = IPW16 + (HAS_LD ? 1 : 0);      // VMEM ops per wave per tile
  static constexpr int XROWS = 32 * WAVES;                  // own rows per workgroup
};

// LDS-DMA plan: per wave slot i the lane-constant source byte offset inside the region's tile, the
// LDS offset inside the ring slot, the region's per-tile stride and its buffer descriptor.
template <int D, typename G>
struct BwdDmaT {
  unsigned voff[G::IPW16];
  unsigned lds_off[G::IPW16];
  unsigned stride[G::IPW16];
  v4u rsrc[G::IPW16];   // the slot's region tensor (head rows 0 .. S-1)
  v4u ld_rsrc;
  QA_DEVICE void init(int wave, int lane, int S, const char* y8a, const char* y8b, const char* tr,
                      const char* tr2, const char* ld) {
#pragma unroll
    for (int i = 0; i < G::IPW16; ++i) {
      int p = wave + G::WAVES * i;
      if (p >= G::INST) p = wave;   // padding slot: re-issue the wave's first piece (same bytes)
      if (p < G::NP8) {
        set_i8(i, G::Y8A, p, lane);
        rsrc[i] = make_rsrc(y8a, (unsigned)S * D);
      } else if (G::TWO && p < 2 * G::NP8) {
        set_i8(i, G::Y8B, p - G::NP8, lane);
        rsrc[i] = make_rsrc(y8b, (unsigned)S * D);
      } else {
        int q = p - (G::TWO ? 2 : 1) * G::NP8;
        const bool second = q >= G::NP16;
        if (second) q -= G::NP16;
        constexpr int NCH = 2 * D / 16, RPI = 64 / NCH;
        const int row = q * RPI + lane / NCH, c = lane % NCH;
        voff[i] = row * 2 * D + 16 * (c ^ t16_sw<D>(row));
        lds_off[i] = (second ? G::TR2 : G::TR) + q * 1024;
        stride[i] = 64 * D;
        rsrc[i] = make_rsrc(second ? tr2 : tr, (unsigned)S * 2 * D);
      }
    }
    if constexpr (G::HAS_LD) ld_rsrc = make_rsrc(ld, (unsigned)S * 8);
  }
  QA_DEVICE void set_i8(int i, int region, int piece, int lane) {
    constexpr int NCH = D / 16, RPI = 64 / NCH;
    const int row = piece * RPI + lane / NCH, c = lane % NCH;
    voff[i] = row * D + 16 * (c ^ i8_sw<D>(row));
    lds_off[i] = region + piece * 1024;
    stride[i] = 32 * D;
  }
  // slot_lds: LDS byte address of the ring slot
  QA_DEVICE void issue(unsigned slot_lds, int t, int lane) const {
#pragma unroll
    for (int i = 0; i < G::IPW16; ++i)
      dma16_buf(rsrc[i], voff[i], (unsigned)t * stride[i], slot_lds + lds_off[i]);
    if constexpr (G::HAS_LD) dma4_buf(ld_rsrc, 4 * lane, (unsigned)t * 256, slot_lds + G::LDO);
  }
};
template <int D, int ROLE>
using BwdDma = BwdDmaT<D, BwdCfg<D, ROLE>>;

// Inline-asm VALU blocks here write only registers tied to their inputs ("+v"), as a precaution:
// hipcc's hazard recogniser does not look inside inline asm, so an asm output placed in a register
// an in-flight MFMA still reads would get no wait states.  A tied register holds a VALU result that
// no MFMA reads, or a copy the compiler made (its own hazard waits included).

// y = RTZ_f32(x * inv + 2^23) = 2^23 + floor(x * inv) for 0 <= x * inv < 2^23 (the f32 spacing is 1
// in [2^23, 2^24)): the truncation of a non-negative quantiser step folded into its multiply, in
// place (y = x on entry).  MODE.FP_ROUND[1:0] (f32) = 3 (toward zero) only around the 16 ops (an
// s_setreg builtin does not order the compiler's FP ops against it).  floor of the exact product:
// differs from trunc(RNE(x * inv)) only when the product lies within half an ulp below an integer.
QA_DEVICE void floor_magic16(float* y, float inv) {
  const float magic = 8388608.0f;
  asm("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 2), 3\n\t"
      "s_nop 1\n\t"
      "v_fma_f32 %0, %0, %16, %17\n\tv_fma_f32 %1, %1, %16, %17\n\t"
      "v_fma_f32 %2, %2, %16, %17\n\tv_fma_f32 %3, %3, %16, %17\n\t"
      "v_fma_f32 %4, %4, %16, %17\n\tv_fma_f32 %5, %5, %16, %17\n\t"
      "v_fma_f32 %6, %6, %16, %17\n\tv_fma_f32 %7, %7, %16, %17\n\t"
      "v_fma_f32 %8, %8, %16, %17\n\tv_fma_f32 %9, %9, %16, %17\n\t"
      "v_fma_f32 %10, %10, %16, %17\n\tv_fma_f32 %11, %11, %16, %17\n\t"
      "v_fma_f32 %12, %12, %16, %17\n\tv_fma_f32 %13, %13, %16, %17\n\t"
      "v_fma_f32 %14, %14, %16, %17\n\tv_fma_f32 %15, %15, %16, %17\n\t"
      "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 2), 0\n\t"
      "s_nop 1"
      : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]),
        "+v"(y[7]), "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]), "+v"(y[12]), "+v"(y[13]),
        "+v"(y[14]), "+v"(y[15])
      : "v"(inv), "s"(magic));
}

// The int8 bytes of 16 integer-valued floats in [-127, 127], packed low to high (byte j of the
// result = x[j]): each conversion writes its byte in place (SDWA dst_sel), 16 instructions instead
// of 16 conversions and 12 byte permutes (tools/ubench/sdwa_probe.hip checks the byte placement).
// Dword w is built in the register of x[4w] (tied, see above).  The four dwords are built
// interleaved, byte b of every dword before byte b + 1: back to back, SDWA partial (PRESERVE) writes
// to one register lose byte 2 (tools/ubench/sdwa_probe.hip: 1012 of 1024 dwords wrong; this
// corrupted dq, tools/ws_records.py) -- a hazard hipcc would have padded around its own code.
QA_DEVICE v4i pack16_i8(const float* x) {
  float r0 = x[0], r1 = x[4], r2 = x[8], r3 = x[12];
#define QA_SDWA(R, A, B, U) \
  "v_cvt_i32_f32_sdwa " R ", " A " dst_sel:BYTE_" B " dst_unused:UNUSED_" U " src0_sel:DWORD\n\t"
  asm(QA_SDWA("%0", "%0", "0", "PAD") QA_SDWA("%1", "%1", "0", "PAD")
      QA_SDWA("%2", "%2", "0", "PAD") QA_SDWA("%3", "%3", "0", "PAD")
      QA_SDWA("%0", "%4", "1", "PRESERVE") QA_SDWA("%1", "%7", "1", "PRESERVE")
      QA_SDWA("%2", "%10", "1", "PRESERVE") QA_SDWA("%3", "%13", "1", "PRESERVE")
      QA_SDWA("%0", "%5", "2", "PRESERVE") QA_SDWA("%1", "%8", "2", "PRESERVE")
      QA_SDWA("%2", "%11", "2", "PRESERVE") QA_SDWA("%3", "%14", "2", "PRESERVE")
      QA_SDWA("%0", "%6", "3", "PRESERVE") QA_SDWA("%1", "%9", "3", "PRESERVE")
      QA_SDWA("%2", "%12", "3", "PRESERVE") QA_SDWA("%3", "%15", "3", "PRESERVE")
      : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3)
      : "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[5]), "v"(x[6]), "v"(x[7]), "v"(x[9]), "v"(x[10]),
        "v"(x[11]), "v"(x[13]), "v"(x[14]), "v"(x[15]));
#undef QA_SDWA
  return v4i{__float_as_int(r0), __float_as_int(r1), __float_as_int(r2), __float_as_int(r3)};
}

// max over |x| of 16 values (v_max3_f32 with abs modifiers)
QA_DEVICE float max16_abs3(const float* x) {
  float m = fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fabsf(x[2]));
#pragma unroll
  for (int i = 3; i < 15; i += 2) m = fmaxf(fmaxf(m, fabsf(x[i])), fabsf(x[i + 1]));
  return fmaxf(m, fabsf(x[15]));
}

// Shapes: the own side has BHx heads of Sx rows; own head bh streams the Ny rows
// starting at row (bh / ydiv) * Ny of the streamed tensors -- dK/dV: the G query heads that share a
// key/value head (Ny = G * Sq, contiguous), dQ: the key/value head of the query head (ydiv = G,
// Ny = Sk).  CAUSAL drops key > query (positions: streamed row mod Smod).
// WS (ROLE_DKV only): also write every quantised dS tile (dS_i8 in this kernel's register order,
// 16 bytes per lane, and its scale s_dS) to the dS workspace that int8_bwd_dqw_kernel reads, so the
// dQ pass does not recompute S, dP, P and dS.  Tile record (query head, q-tile, key tile) =
// ((bh_q * nqt + qt) * nkt + kt): 1024 bytes in ds8, one float in sds.
// Diagnostic build only (-DQA_DKV_STAMP=1, tools/dkv_stamps.py): s_memrealtime stamps (100 MHz) of
// every fused dK+dV workgroup with records -- entry, end of the prologue, end of the tile loop, exit
// -- written by lane 0 of wave 0 with vector stores to a buffer of their own that no other code reads.
#ifndef QA_DKV_STAMP
#define QA_DKV_STAMP 0
#endif
#if QA_DKV_STAMP
__device__ unsigned long long g_dkv_stamp[4096][4];
#define DKV_STAMP(k)                                                                            \
  do {                                                                                          \
    if (ROLE == ROLE_DKV && WS && threadIdx.x == 0 && blockIdx.x < 4096)                         \
      g_dkv_stamp[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                            \
  } while (0)
#else
#define DKV_STAMP(k) do { } while (0)
#endif
template <int D, int ROLE, bool CAUSAL = false, bool WS = false>
__global__ __launch_bounds__((64 * BwdCfg<D, ROLE>::WAVES), (8 / BwdCfg<D, ROLE>::WAVES))
void int8_bwd_kernel(
    const int8_t* __restrict__ x8a, const int8_t* __restrict__ x8b, const _Float16* __restrict__ sxa,
    const _Float16* __restrict__ sxb, const int8_t* __restrict__ y8a, const int8_t* __restrict__ y8b,
    const __bf16* __restrict__ ytr, const __bf16* __restrict__ ytr2, const float2* __restrict__ yld,
    const _Float16* __restrict__ sya, const _Float16* __restrict__ syb,
    const float2* __restrict__ xld, _Float16* __restrict__ out, _Float16* __restrict__ out2, int BH,
    int Sx, int Ny, int ydiv, int Smod, float qks, float sms, int8_t* __restrict__ ds8,
    float* __restrict__ sds) {
  using C = I8BwdCfg<D>;
  using G = BwdCfg<D, ROLE>;
  constexpr bool TWO = G::TWO;
  static_assert(!WS || ROLE == ROLE_DKV, "the dS workspace is written by the fused dK+dV kernel");
  DKV_STAMP(0);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nxb = (Sx + G::XROWS - 1) / G::XROWS;
  int bh, xt;
  if constexpr (CAUSAL && ROLE == ROLE_DKV && QA_DKV_HG > 0)
    xcd_remap_lpt_grouped(blockIdx.x, nxb, BH, false, QA_DKV_HG, bh, xt);
  else if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nxb, BH, ROLE == ROLE_DQ, bh, xt);
  else xcd_remap(blockIdx.x, nxb, BH, bh, xt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int x0 = xt * G::XROWS + wave * 32;
  const bool active = x0 < Sx;
  const long hrow = (long)bh * Sx;                 // own rows
  const long yrow = (long)(bh / ydiv) * Ny;        // streamed rows
  // causal dQ: key tiles past the workgroup's last query are masked for all of its rows
  const int nt = (CAUSAL && ROLE == ROLE_DQ) ? min(Ny / 32, (xt * G::XROWS + G::XROWS) / 32) : Ny / 32;
  // causal dK/dV: query tiles before the workgroup's first key are masked for all of its rows
  // (P = 0 exactly, so skipping them is exact); tiles t0 .. nt-1 are visited
  const int t0 = (CAUSAL && ROLE != ROLE_DQ && Ny == Smod) ? min(nt, (xt * G::XROWS) / 32) : 0;

  BwdDma<D, ROLE> dma;
  dma.init(wave, lane, Ny, reinterpret_cast<const char*>(y8a + yrow * D),
           reinterpret_cast<const char*>(y8b + yrow * D), reinterpret_cast<const char*>(ytr + yrow * D),
           reinterpret_cast<const char*>(ytr2 + yrow * D), reinterpret_cast<const char*>(yld + yrow));
  const unsigned smem_lds = lds_addr(smem);
#pragma unroll
  for (int i = 0; i < G::NSLOT - 1; ++i)
    dma.issue(smem_lds + ((t0 + i) % G::NSLOT) * G::SLOT, min(t0 + i, nt - 1), lane);
  // per-tile scales of the streamed side, once, in LDS (a global load inside the loop would make
  // hipcc wait vmcnt for the in-flight LDS-DMA)
  _Float16* sc_lds = reinterpret_cast<_Float16*>(smem + G::NSLOT * G::SLOT);
  for (int i = tid; i < nt; i += 64 * G::WAVES) {
    sc_lds[i] = sya[yrow / 32 + i];
    sc_lds[nt + i] = syb[yrow / 32 + i];
  }

  // own-side int8 fragments (B operands): lane holds X[x0 + c32][32s + 16h .. +16]
  v4i xa[C::NKS8], xb[C::NKS8];
  float sxaw = 0.f, sxbw = 0.f, lsex = 0.f, Dx = 0.f;
  if (active) {
    const long r = hrow + x0 + c32;
#pragma unroll
    for (int s = 0; s < C::NKS8; ++s) {
      xa[s] = *reinterpret_cast<const v4i*>(x8a + r * D + 16 * h + 32 * s);
      if constexpr (TWO) xb[s] = *reinterpret_cast<const v4i*>(x8b + r * D + 16 * h + 32 * s);
    }
    sxaw = (float)sxa[(hrow + x0) / 32];
    sxbw = (float)sxb[(hrow + x0) / 32];
    if constexpr (!G::HAS_LD) {
      const float2 v = xld[r];
      lsex = v.x;
      Dx = v.y;
    }
  }
  // lane-constant LDS offsets: int8 A-operand rows, tr-image A-operand (per 32-wide d block)
  int roff[C::NKS8], troff[C::NDB];
#pragma unroll
  for (int s = 0; s < C::NKS8; ++s) roff[s] = c32 * D + 16 * ((2 * s + h) ^ i8_sw<D>(c32));
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int row = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      troff[b] = row * 2 * D + 16 * ((d / 8) ^ t16_sw<D>(row)) + (d % 8) * 2;
    }
  }
  v16f acc[C::NDB], acc2[ROLE == ROLE_DKV ? C::NDB : 1];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) acc[b] = v16f{};
  if constexpr (ROLE == ROLE_DKV) {
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) acc2[b] = v16f{};
  }

  auto slot = [&](int t) -> const char* { return smem + (t % G::NSLOT) * G::SLOT; };
  // int8 products of tile t: S (and dP)
  auto products = [&](int t, v16i& sa, v16i& pa) {
    const char* base = slot(t);
    sa = v16i{};
    pa = v16i{};
#pragma unroll
    for (int s = 0; s < C::NKS8; ++s) {
      sa = mfma_i8(*reinterpret_cast<const v4i*>(base + G::Y8A + roff[s]), xa[s], sa);
      if constexpr (TWO) pa = mfma_i8(*reinterpret_cast<const v4i*>(base + G::Y8B + roff[s]), xb[s], pa);
    }
  };
  // fp32 P and/or dS of tile t.  maskc (std::true_type / false_type): whether the causal mask is
  // compiled in -- false_type for tiles past the workgroup's diagonal band, where no score is masked
  // (the same values: the mask changes nothing there)
  auto values = [&](int t, const v16i& sa, const v16i& pa, float* P, float* dS, auto maskc) {
    constexpr bool MASK = CAUSAL && decltype(maskc)::value;
    // causal: position of the tile's first streamed row; the mask is applied only on tiles that
    // cross this wave's diagonal (the streamed side is queries for dK/dV, keys for dQ)
    const int y0 = (32 * t) % Smod;
    const bool diag = MASK && (ROLE == ROLE_DQ ? (y0 + 31 > x0) : (x0 + 31 > y0));
    // c1 = sq*(sk*qks), c2 = sdO*sv with the streamed / own roles of each kernel
    const float sy_a = (float)sc_lds[t], sy_b = (float)sc_lds[nt + t];
    float c1, c2;
    if constexpr (ROLE == ROLE_DQ) {
      c1 = sxaw * (sy_a * qks);
      c2 = sxbw * sy_b;
    } else {
      c1 = sy_a * (sxaw * qks);
      c2 = sy_b * sxbw;
    }
    // key > query as one compare per score against an immediate: dd = key - (first query of the
    // lane's row group), INT_MIN off the diagonal tiles (nothing masked there)
    // (the lane's c32 - 4h is re-derived from the lane id here, two mbcnt and two bit ops, rather
    // than kept live: at 256 VGPRs the causal dK+dV kernels otherwise spill it and reload it from
    // scratch on every tile)
    const int ln = __lane_id();
    const int lane_rel = (ln & 31) - 4 * (ln >> 5);   // c32 - 4h
    const int dd = !diag ? INT_MIN
                         : (ROLE == ROLE_DQ ? (y0 - x0) - lane_rel : (x0 - y0) + lane_rel);
    if constexpr (G::HAS_LD) {
      const float* ld = reinterpret_cast<const float*>(slot(t) + G::LDO);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f a = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h));
        const v4f b = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h) + 4);
        const float lse_r[4] = {a[0], a[2], b[0], b[2]};
        const float d_r[4] = {a[1], a[3], b[1], b[3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g + j;
          float p = exp2_f32(fmaf((float)sa[i], c1, -lse_r[j]));
          if (MASK && dd > 8 * g + j) p = 0.f;   // key > query: x0 + c32 > y0 + 8g + 4h + j
          if constexpr (G::WANT_P) P[i] = p;
          if constexpr (G::WANT_DS) dS[i] = p * fmaf((float)pa[i], c2, -d_r[j]);
        }
      }
    } else {
      // per-lane row stats; the same operations as the dK/dV kernels' (so every kernel quantises a
      // dS tile to the same dS_i8 and scale, and the dS workspace path is bit-identical to this one)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = exp2_f32(fmaf((float)sa[i], c1, -lsex));
        // key > query: y0 + (i & 3) + 8 (i >> 2) + 4h > x0 + c32
        if (MASK && dd > -((i & 3) + 8 * (i >> 2))) p = 0.f;
        dS[i] = p * fmaf((float)pa[i], c2, -Dx);
      }
    }
  };
  // per-tile quantisation of X into the two bf16 B operands, scaled by so (the other operand's
  // per-tile scale)
  // xmax: the tile's max |X| (wave_max_nonneg of max16_abs3)
  auto quantise_m = [&](const float* X, float so, v8bf* op, float xmax) {
    const float sx = xmax * (1.0f / 127.0f);
    const float inv = xmax > 0.f ? 127.0f * __builtin_amdgcn_rcpf(xmax) : 0.f;
    quant_operand(X, inv, sx * so, op);
  };
  auto quantise = [&](const float* X, float so, v8bf* op) {
    quantise_m(X, so, op, wave_max_nonneg(max16_abs3(X)));
  };
  // the P operand (P >= 0): trunc = floor, folded into the multiply (floor_magic16), and
  // q * c = fma(2^23 + q, c, -2^23 c) exactly (2^23 c is exact): 2 ops per value instead of 3
  auto quantise_p = [&](const float* X, float so, v8bf* op, float xmax) {
    const float sx = xmax * (1.0f / 127.0f);
    const float inv = xmax > 0.f ? 127.0f * __builtin_amdgcn_rcpf(xmax) : 0.f;
    const float c = sx * so;
    const float nc = -8388608.0f * c;
    float y[16];
#if QA_BWD_PACK_ASM
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = X[i];
    floor_magic16(y, inv);
#else
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = __builtin_truncf(X[i] * inv) + 8388608.0f;
#endif
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      v4u w;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i0 = 8 * s + 2 * j;
        w[j] = pk_bf16(fmaf(y[i0], c, nc), fmaf(y[i0 + 1], c, nc));
      }
      op[s] = __builtin_bit_cast(v8bf, w);
    }
  };
  auto tr_load = [&](int t, int region, v8bf* ta) {
    const char* base = slot(t) + region;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) {
        const char* a = base + troff[b] + 16 * s * 2 * D;
        ta[s * C::NDB + b] = __builtin_bit_cast(v8bf, ds_read_tr16_x2(a, a + 8 * 2 * D));
      }
  };
  // Timing-only cost model (A/B builds, -DQA_DKV_I8DV_COST=1; results are wrong): dV on the int8
  // MFMA as the reference's hl.dot(P_i8^T, dO_i8) (int8:375-378) -- 4 v_mfma_i32_32x32x32_i8 from a
  // biased seed and the per-tile dequantisation of the 64 accumulator elements per lane -- in place
  // of the 8 bf16 MFMAs of the folded-scale operand; operands are stand-ins of the same registers.
  auto accumulate_i8cost = [&](v16f* ac, const v8bf* ta, const v8bf* op, float c) {
    v16i seed;
#pragma unroll
    for (int i = 0; i < 16; ++i) seed[i] = KMAG_BITS;
    // one d block at a time (a 64-register int32 product beside the fp32 accumulators spills)
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const v16i pacc = mfma_i8(__builtin_bit_cast(v4i, ta[b]), __builtin_bit_cast(v4i, op[0]), seed);
#pragma unroll
      for (int r = 0; r < 16; ++r) ac[b][r] = fmaf(__int_as_float(pacc[r]), c, ac[b][r]);
    }
  };
  auto accumulate = [&](v16f* ac, const v8bf* ta, const v8bf* op) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) ac[b] = mfma_bf16(ta[s * C::NDB + b], op[s], ac[b]);
  };
  // scale of the other operand of the accumulating product: DV/DKV-P: dO of the q tile (syb);
  // DK/DKV-dS: q of the q tile (sya); DQ: k of the k tile (sya)
  auto so_p = [&](int t) { return (float)sc_lds[nt + t]; };
  auto so_ds = [&](int t) { return (float)sc_lds[t]; };
  // dS workspace of this key/value head's G query heads: records (bh*G*nqt + t) * nkt + kt for the
  // streamed tile t (= g * nqt + qt) -- one contiguous region per key/value head (< 4 GiB)
  const long ws_first = WS ? (long)bh * (Ny / 32) * (Sx / 32) : 0;
  const int ws_nrec = WS ? (Ny / 32) * (Sx / 32) : 0;
  const __amdgpu_buffer_rsrc_t ws_rsrc =
      __builtin_amdgcn_make_buffer_rsrc(ds8 + ws_first * 1024, 0, ws_nrec * 1024, 0x00020000);
  // the tile scales s_dS stay in LDS until the loop ends (one VMEM store per tile, not two)
  float* sds_lds = reinterpret_cast<float*>(smem + G::NSLOT * G::SLOT +
                                            ((2 * nt * 2 + 15) / 16) * 16);
  // dS quantisation (the dK operand, as quantise()) that also emits the workspace record of tile t:
  // the 16 dS_i8 of this lane packed in index order, and s_dS (lane 0).  Two VMEM stores per tile,
  // counted by the ring waits below (WS_OPS).
  auto quantise_ds = [&](const float* X, int t, v8bf* op, float xmax) {
    if constexpr (!WS) {
      quantise_m(X, so_ds(t), op, xmax);
    } else {
      const float sx = xmax * (1.0f / 127.0f);
      const float inv = xmax > 0.f ? 127.0f * __builtin_amdgcn_rcpf(xmax) : 0.f;
      const float c = sx * so_ds(t);
      float q[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) q[i] = __builtin_truncf(X[i] * inv);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        v4u w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = pk_bf16(q[8 * s + 2 * j] * c, q[8 * s + 2 * j + 1] * c);
        op[s] = __builtin_bit_cast(v8bf, w);
      }
#if QA_BWD_PACK_ASM
      const v4i bytes = pack16_i8(q);
#else
      v4i bytes;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const unsigned lo = __builtin_amdgcn_perm((unsigned)(int)q[4 * d + 1], (unsigned)(int)q[4 * d],
                                                  0x0c0c0400u);
        const unsigned hi = __builtin_amdgcn_perm((unsigned)(int)q[4 * d + 3], (unsigned)(int)q[4 * d + 2],
                                                  0x0c0c0400u);
        bytes[d] = (int)__builtin_amdgcn_perm(hi, lo, 0x05040100u);
      }
#endif
      // record of (query head bh*G + t/nqt, q-tile t%nqt, key tile x0/32), relative to this key/value
      // head's first record (ws_rsrc / sc_rsrc)
      const int nqt = Smod / 32, nkt = Sx / 32;
      const unsigned rel = (unsigned)(t * nkt + x0 / 32);
      // The tile offset goes in the VGPR offset with soffset = 0: hipcc pads a VALU write of the
      // data registers of a > 64-bit buffer store (2 wait states) only when soffset is not a
      // register, while on gfx950 the hazard holds either way.  With the offset in an SGPR the
      // second instruction after the store (a v_and into the register of dword 0) overwrote the data
      // before the store read it: dword 0 of some records of the last query tile came out wrong,
      // run-dependently, at D = 64 (tools/nondet_probe3.py; tests/test_gpu_int8_ext.py::
      // test_int8_bwd_ws_long_d64; tests/test_isa.py checks the emitted code).
      // (slot of lane l: l ^ 4(l >> 5), so the dQ pass's transposed reads of two slot halves fall on
      // different banks, int8_bwd_dqw_kernel)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, bytes), ws_rsrc,
                                             16 * (lane ^ ((lane >> 5) << 2)) + (int)(rel * 1024u), 0, 0);
      (void)nqt;
      if (lane == 0) sds_lds[wave * nt + t] = sx;   // written out after the loop
    }
  };
  // VMEM operations per tile besides the ring DMA (the workspace store of an active wave)
  constexpr int WS_OPS = WS ? 1 : 0;

  vmem_drain();
  __syncthreads();
  DKV_STAMP(1);
  if constexpr (G::PIPE) {
    float X[16];
    if (active && t0 < nt) {
      v16i sa, pa;
      products(t0, sa, pa);
      values(t0, sa, pa, X, X, std::true_type{});
    }
    for (int t = t0; t < nt; ++t) {
      // tile t+1 landed (later tiles may be in flight); the slot of tile t-1 is free
      ring_wait_barrier<(G::NSLOT - 3) * G::IPW>();
      dma.issue(smem_lds + ((t + G::NSLOT - 1) % G::NSLOT) * G::SLOT,
                min(t + G::NSLOT - 1, nt - 1), lane);
      if (active) {
        const int tn = min(t + 1, nt - 1);
        v8bf ta[2 * C::NDB];
        tr_load(t, G::TR, ta);
        v16i sa, pa;
        products(tn, sa, pa);
        v8bf op[2];
        if constexpr (ROLE == ROLE_DV) quantise_p(X, so_p(t), op, wave_max_nonneg(max16_abs3(X)));
        else quantise(X, so_ds(t), op);
        accumulate(acc, ta, op);
        values(tn, sa, pa, X, X, std::true_type{});
      }
    }
  } else {
    // Fused dK+dV.  Causal without grouped heads (the streamed rows are one query head): the tiles
    // t0 .. t0 + WAVES - 1 hold every wave's diagonal; past this band no score of the workgroup is
    // masked, and those tiles run with the mask compiled out (bit-identical, ~36 fewer vector
    // instructions per tile-wave).  Grouped heads stream the group's query heads one after another,
    // so their diagonals recur: masked throughout.
    const int tb = !CAUSAL ? t0 : (Ny == Smod ? min(nt, t0 + G::WAVES) : nt);
    // (A/B) static priority for one half of the workgroup (MI355X_MICROARCH "Two waves per SIMD",
    // item 4): QA_DKV_PRIO = 1 raises waves 4-7 (the staggered half), 2 waves 0-3
    if (QA_DKV_PRIO == 1 && wave >= G::WAVES / 2) __builtin_amdgcn_s_setprio(1);
    if (QA_DKV_PRIO == 2 && wave < G::WAVES / 2) __builtin_amdgcn_s_setprio(1);
    if (QA_DKV_PIPE || (QA_DKV_STAGGER && wave >= G::WAVES / 2)) {
      // DKV pipelined: carry the quantised bf16 operands of tile t (16 VGPRs) into iteration t, whose
      // int8 products for tile t+1 are issued first and whose fp32 values of t+1 are computed beside
      // the bf16 MFMAs of tile t
      v8bf opS[2], opP[2];
      if (active && t0 < nt) {
        v16i sa, pa;
        products(t0, sa, pa);
        float P[16], dS[16];
        values(t0, sa, pa, P, dS, std::true_type{});
        float mS = max16_abs3(dS), mP = max16_abs3(P);
        wave_max2_nonneg(mS, mP);   // (the two tile maxima in one interleaved reduction)
        quantise_ds(dS, t0, opS, mS);
        quantise_p(P, so_p(t0), opP, mP);
      }
      auto iter = [&](int t, auto maskc) {
        // tile t+1 landed: younger than its DMA are the workspace stores of tile t-1, the DMA of
        // tile t+2 and the stores of tile t
        if (active) ring_wait_barrier<(G::NSLOT - 3) * G::IPW + 2 * WS_OPS>();
        else ring_wait_barrier<(G::NSLOT - 3) * G::IPW>();
        dma.issue(smem_lds + ((t + G::NSLOT - 1) % G::NSLOT) * G::SLOT,
                  min(t + G::NSLOT - 1, nt - 1), lane);
        if (active) {
          const int tn = min(t + 1, nt - 1);
          v16i sa, pa;
          products(tn, sa, pa);
          v8bf ta[2 * C::NDB];
          tr_load(t, G::TR, ta);
          accumulate(acc, ta, opS);          // dK += q^T dS
          tr_load(t, G::TR2, ta);
#if QA_DKV_I8DV_COST
          accumulate_i8cost(acc2, ta, opP, so_p(t));
#else
          accumulate(acc2, ta, opP);         // dV += dO^T P
#endif
          float P[16], dS[16];
          values(tn, sa, pa, P, dS, maskc);  // (tile t+1 of the last band iteration: mask-free anyway)
          float mS = max16_abs3(dS), mP = max16_abs3(P);
          wave_max2_nonneg(mS, mP);   // (the two tile maxima in one interleaved reduction)
          quantise_ds(dS, tn, opS, mS);
          quantise_p(P, so_p(tn), opP, mP);
        }
      };
      int t = t0;
      for (; t < tb; ++t) iter(t, std::true_type{});
      for (; t < nt; ++t) iter(t, std::false_type{});
    } else {
      auto iter = [&](int t, auto maskc) {
        // tile t landed (t+1, t+2 may be in flight); the slot of tile t-1 is free.  With the stagger
        // the other half of the workgroup reads tile t+1 after this barrier: wait for it too.
        // (the workspace stores of an active wave, WS_OPS per tile, sit between the DMAs)
        if (active)
          ring_wait_barrier<(G::NSLOT - (QA_DKV_STAGGER ? 3 : 2)) * G::IPW +
                            (QA_DKV_STAGGER ? 2 : 3) * WS_OPS>();
        else
          ring_wait_barrier<(G::NSLOT - (QA_DKV_STAGGER ? 3 : 2)) * G::IPW>();
        dma.issue(smem_lds + ((t + G::NSLOT - 1) % G::NSLOT) * G::SLOT,
                  min(t + G::NSLOT - 1, nt - 1), lane);
        if (active) {
          v16i sa, pa;
          products(t, sa, pa);
          float P[16], dS[16];
          values(t, sa, pa, P, dS, maskc);
          v8bf opS[2], opP[2];
          float mS = max16_abs3(dS), mP = max16_abs3(P);
          wave_max2_nonneg(mS, mP);   // (the two tile maxima in one interleaved reduction)
          quantise_ds(dS, t, opS, mS);
          quantise_p(P, so_p(t), opP, mP);
          v8bf ta[2 * C::NDB];
          tr_load(t, G::TR, ta);
          accumulate(acc, ta, opS);          // dK += q^T dS
          tr_load(t, G::TR2, ta);
#if QA_DKV_I8DV_COST
          accumulate_i8cost(acc2, ta, opP, so_p(t));
#else
          accumulate(acc2, ta, opP);         // dV += dO^T P
#endif
        }
      };
      int t = t0;
      for (; t < tb; ++t) iter(t, std::true_type{});
      for (; t < nt; ++t) iter(t, std::false_type{});
    }
  }
  vmcnt_wait_all();
  DKV_STAMP(2);
  if (!active) return;
  if constexpr (WS) {   // this wave's s_dS column: record (t, x0/32) of the key/value head
    const int nkt = Sx / 32;
    for (int t = t0 + lane; t < nt; t += 64) sds[ws_first + (long)t * nkt + x0 / 32] = sds_lds[wave * nt + t];
  }
  const long r = hrow + x0 + c32;
  auto store = [&](const v16f* ac, float osc, _Float16* dst) {
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        v4h w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (_Float16)(ac[b][4 * g + j] * osc);
        *reinterpret_cast<v4h*>(dst + r * D + 32 * b + 8 * g + 4 * h) = w;
      }
    }
  };
  store(acc, ROLE == ROLE_DV ? 1.0f : sms, out);
  if constexpr (ROLE == ROLE_DKV) store(acc2, 1.0f, out2);
#if QA_DKV_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  DKV_STAMP(3);
#endif
}


// ------------------------------------------------------------- dQ from the dS workspace (WS)
// The fused dK+dV kernel (WS) leaves every quantised dS tile in the workspace: dS_i8 in its own
// register order (key on the lane: lane l holds key l%32 and the 16 queries 8(i/4) + 4(l/32) + i%4,
// byte i) and the tile scale s_dS.  Here a wave owns 32 queries and streams 32-key tiles: the k
// image through the LDS ring as in int8_bwd_kernel<ROLE_DQ>, its own 1 KiB dS record of the tile
// beside it.  One v_mfma_i32_32x32x32_i8 against a permutation matrix P brings the record into the
// dQ order (query on the lane, keys 8(i/4) + 4(l/32) + i%4: C = A P with A = the record, rows =
// keys), and the tile then takes exactly the operand / MFMA sequence of the ROLE_DQ kernel:
// op = bf16(dS_i8 * (s_dS * sk)), dQ^T += K^T op.  The result is bit-identical to that kernel's,
// which recomputes S, dP, P and dS (2 int8 MFMA chains, ~150 VALU per tile) where this pass spends
// one int8 MFMA and ~40 VALU.
#ifndef QA_DQW_WAVES
#define QA_DQW_WAVES 8
#endif
// Timing-only diagnostics (results wrong): every tile's record load reads the wave's first record
// (bit 1: no HBM record stream), every k-image load reads the head's first key tile (bit 2); no
// record DMA at all (bit 4), no k-image DMA at all (bit 8)
#ifndef QA_DQW_DIAG
#define QA_DQW_DIAG 0
#endif
#ifndef QA_DQW_NT
#define QA_DQW_NT 1
#endif
// QA_DQW_TR8 (A/B): the record read as two ds_read_b64_tr_b8 straight into dQ order (1) instead of
// one 16-B read and the permutation MFMA (0).  Bit-identical dq, 92 instead of 115 VGPRs, one MFMA
// fewer per tile-wave -- and measured no faster: 162-171 against 156-165 us per 32-head chunk at
// config 3 (profiles/r05_dqw_tr8_ab.log; the kernel is bound by the record stream).
#ifndef QA_DQW_TR8
#define QA_DQW_TR8 0
#endif
#ifndef QA_DQW_NSLOT
#define QA_DQW_NSLOT 4
#endif
// The dK+dV kernel (8 waves) writes records only for q-tiles >= its workgroup's first key tile,
// and this kernel reads every key tile up to its workgroup's last query tile for all of its waves:
// with more than 8 waves per workgroup the first ones would read records never written (causal).
#ifndef QA_DQW_ALLOW_WIDE   // (A/B, non-causal timing only: wider workgroups break the causal records)
static_assert(QA_DQW_WAVES <= 8, "dQ-from-records workgroups may not exceed the dK+dV kernel's 8 waves");
#endif
template <int D>
struct DqwCfg {
  static constexpr int WAVES = QA_DQW_WAVES;
  static constexpr int T16 = 64 * D;               // bf16 k image of a 32-key tile (L2-resident)
  static constexpr int NSLOT = QA_DQW_NSLOT;       // k image ring: NSLOT - 1 tiles ahead
#ifdef QA_DQW_RSLOT
  static constexpr int RSLOT = QA_DQW_RSLOT;
#else
  static constexpr int RSLOT = WAVES >= 16 ? 4 : WAVES == 8 ? 5 : 10;   // record ring (HBM stream)
#endif
  static constexpr int REC = WAVES * 1024;         // the waves' dS records of one tile
  static constexpr int RBASE = NSLOT * T16;
  static constexpr int NP16 = T16 / 1024;
  // k image pieces per wave per tile; with more waves than pieces the extra waves re-issue a
  // piece (the same bytes to the same place), so every wave issues IPK + 1 DMAs per tile
  static constexpr int IPK = (NP16 + WAVES - 1) / WAVES;
  // the pipelined loop reads tile t+1's record with tile t's k image: records run >= 1 tile ahead
  static_assert(RSLOT - 1 >= NSLOT, "record ring must run ahead of the k image ring");
};

template <int D, bool CAUSAL>
__global__ __launch_bounds__(64 * QA_DQW_WAVES, QA_DQW_WAVES >= 16 ? 4 : 2) void int8_bwd_dqw_kernel(
    const int8_t* __restrict__ ds8, const float* __restrict__ sds, const __bf16* __restrict__ kbf,
    const _Float16* __restrict__ sk, _Float16* __restrict__ dq, int BH, int Sq, int Sk, int G,
    float sms) {
  using C = I8BwdCfg<D>;
  using W = DqwCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (Sq + 32 * W::WAVES - 1) / (32 * W::WAVES);
  int bh, qb;
  if constexpr (CAUSAL && QA_DQW_HG > 0) xcd_remap_lpt_grouped(blockIdx.x, nqb, BH, true, QA_DQW_HG, bh, qb);
  else if constexpr (CAUSAL) xcd_remap_lpt(blockIdx.x, nqb, BH, true, bh, qb);
  else xcd_remap(blockIdx.x, nqb, BH, bh, qb);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qb * 32 * W::WAVES + wave * 32;
  const bool active = q0 < Sq;
  const int nqt = Sq / 32, nkt = Sk / 32;
  const long kv_row0 = (long)(bh / G) * Sk;
  // causal: key tiles past the workgroup's last query are all zero for its rows (as ROLE_DQ)
  const int nt = CAUSAL ? min(nkt, (qb * 32 * W::WAVES + 32 * W::WAVES) / 32) : nkt;
  const long rec0 = ((long)bh * nqt + (active ? q0 / 32 : 0)) * nkt;   // this wave's first record

  // DMA plan: pieces of the k image (swizzled rows, as BwdDma's TR region), and the own record
  unsigned kvoff[W::IPK], klds[W::IPK];
  v4u krsrc[W::IPK];
#pragma unroll
  for (int i = 0; i < W::IPK; ++i) {
    int pc = wave + W::WAVES * i;
    if (pc >= W::NP16) pc = wave % W::NP16;
    constexpr int NCH = 2 * D / 16, RPI = 64 / NCH;
    const int row = pc * RPI + lane / NCH, c = lane % NCH;
    kvoff[i] = row * 2 * D + 16 * (c ^ t16_sw<D>(row));
    klds[i] = pc * 1024;
    krsrc[i] = make_rsrc(kbf + kv_row0 * D, (unsigned)Sk * 2 * D);
  }
  // an inactive wave's descriptor has no records: its loads return zeros, nothing is read
  const v4u rrsrc = make_rsrc(ds8 + rec0 * 1024, active ? (unsigned)nkt * 1024u : 0u);
  const unsigned smem_lds = lds_addr(smem);
  auto issue_k = [&](int t) {
    const unsigned sl = smem_lds + (t % W::NSLOT) * W::T16;
#pragma unroll
    for (int i = 0; i < W::IPK; ++i)
      if (!(QA_DQW_DIAG & 8)) dma16_buf(krsrc[i], kvoff[i], (QA_DQW_DIAG & 2) ? 0u : (unsigned)min(t, nt - 1) * 64u * D, sl + klds[i]);
  };
  auto issue_r = [&](int t, int rs) {   // record of tile t into ring slot rs; read once: non-temporal
    if (QA_DQW_DIAG & 4) return;
#if QA_DQW_NT
    dma16_buf_nt(rrsrc, 16u * lane, (QA_DQW_DIAG & 1) ? 0u : (unsigned)min(t, nt - 1) * 1024u,
#else
    dma16_buf(rrsrc, 16u * lane, (QA_DQW_DIAG & 1) ? 0u : (unsigned)min(t, nt - 1) * 1024u,
#endif
              smem_lds + W::RBASE + rs * W::REC + wave * 1024);
  };
#pragma unroll
  for (int i = 0; i < W::NSLOT - 1; ++i) issue_k(i);
#pragma unroll
  for (int i = 0; i < W::RSLOT - 1; ++i) issue_r(i, i);
  // per-tile operand scales s_dS * sk of each wave's records, once, in LDS (0 for an inactive
  // wave, whose zero records then give zero operands; one padding float after the last wave's for
  // the discarded operand of the loop's last iteration)
  float* c_lds = reinterpret_cast<float*>(smem + W::RBASE + W::RSLOT * W::REC);
  for (int i = lane; i < nt; i += 64) c_lds[wave * nkt + i] = active ? sds[rec0 + i] * (float)sk[kv_row0 / 32 + i] : 0.f;

#if QA_DQW_TR8
  // ds_read_b64_tr_b8 of the record (per 16-lane group: lane 2j+p reads bytes 8p..8p+7 of row j,
  // lane i receives byte i of the 8 rows): rows = the record slots (key on the row) of the 8 keys of
  // this lane's B-operand k-step, in the k order of the k image's A operand (key 16s + 8(j >> 2) +
  // 4h + (j & 3)); the slot half (lane >> 4) & 1 picks the queries: lane l receives query
  // qcol(l & 31) = 8((c & 15) >> 2) + 4(c >> 4) + (c & 3) of the record's byte order, and the
  // epilogue stores column c to that row.  No permutation MFMA; the same products in the same order.
  int rtr;
  {
    const int j = (lane & 15) >> 1;
    const int hq = (lane >> 4) & 1;   // record slot key + 32 hq, stored at (key ^ 4hq) + 32 hq
    rtr = 16 * (((8 * (j >> 2) + 4 * h + (j & 3)) ^ (4 * hq)) + 32 * hq) + 8 * (lane & 1);
  }
#else
  // permutation operand: byte i of lane l is 1 iff query 8(i/4) + 4(l/32) + i%4 is this lane's
  // column l%32 (one byte in the lane half that holds it)
  v4i perm = {0, 0, 0, 0};
  if (((c32 >> 2) & 1) == h) {
    const int i = 4 * (c32 >> 3) + (c32 & 3);
    perm[i >> 2] = 1 << (8 * (i & 3));
  }
#endif
  int troff[C::NDB];
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int row = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      troff[b] = row * 2 * D + 16 * ((d / 8) ^ t16_sw<D>(row)) + (d % 8) * 2;
    }
  }
  v16f acc[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) acc[b] = v16f{};

  // the bf16 operand of tile t (its record in ring slot rs): the record brought into dQ order by
  // the permutation MFMA (exact integers), scaled by s_dS * sk
  auto make_op = [&](int t, int rs, v8bf* op) {
    const float c = c_lds[wave * nkt + t];
#if QA_DQW_TR8
    const char* rb = smem + W::RBASE + rs * W::REC + wave * 1024 + rtr;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const v2i x = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
          (__attribute__((address_space(3))) v2i*)(rb + 256 * s));   // keys 16s .. 16s + 15
      v4u w;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int wd = x[j >> 1], sh = 16 * (j & 1);
        w[j] = pk_bf16((float)(signed char)(wd >> sh) * c, (float)(signed char)(wd >> (sh + 8)) * c);
      }
      op[s] = __builtin_bit_cast(v8bf, w);
    }
#else
    const v4i rec = *reinterpret_cast<const v4i*>(smem + W::RBASE + rs * W::REC + wave * 1024 +
                                                  16 * (lane ^ ((lane >> 5) << 2)));
    const v16i x = mfma_i8(rec, perm, v16i{});   // dS_i8 in dQ order (exact integers)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      v4u w;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = pk_bf16((float)x[8 * s + 2 * j] * c, (float)x[8 * s + 2 * j + 1] * c);
      op[s] = __builtin_bit_cast(v8bf, w);
    }
#endif
  };

  vmem_drain();
  __syncthreads();
  // Software-pipelined by one tile: the operand of tile t+1 (record read, permutation MFMA, 16
  // conversions) is formed beside the 8 bf16 MFMAs of tile t, so a wave's MFMA chain does not wait
  // on its own VALU chain.  Same operations as the unpipelined order: dq is bit-identical.
  // Every wave runs the loop (an inactive one on zero records and scales, stored nowhere), and the
  // loop is unrolled by the record ring's RSLOT with its slots as constants, so the tile step has no
  // branch and no modulo of the ring index.
  v8bf op[2];
  make_op(0, 0, op);
  if (QA_DQW_PRIO && wave >= W::WAVES / 2) __builtin_amdgcn_s_setprio(1);   // (A/B, as QA_DKV_PRIO)
  // tile t; rs_next = (t + 1) % RSLOT, rs_issue = (t + RSLOT - 1) % RSLOT
  auto step = [&](int t, int rs_next, int rs_issue) {
    // tile t's k image and tile t+1's record landed: with RSLOT - 1 = NSLOT both were issued three
    // iterations ago, and younger than them are the k + record DMAs of the two iterations since
    // (records more than one tile ahead of the k image: tile t's k image binds, and its
    // iteration's record DMA is younger)
    ring_wait_barrier<(W::RSLOT - 1 > W::NSLOT ? 1 : 0) + (W::NSLOT - 2) * (W::IPK + 1)>();
    issue_k(t + W::NSLOT - 1);
    issue_r(t + W::RSLOT - 1, rs_issue);
    const char* kb = smem + (t % W::NSLOT) * W::T16;
    v8bf ta[2 * C::NDB];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) {
        const char* a = kb + troff[b] + 16 * s * 2 * D;
        ta[s * C::NDB + b] = __builtin_bit_cast(v8bf, ds_read_tr16_x2(a, a + 8 * 2 * D));
      }
    // (the last iteration forms an operand from slot nt % RSLOT and the scale after the wave's
    // last: discarded)
    v8bf opn[2];
    make_op(t + 1, rs_next, opn);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) acc[b] = mfma_bf16(ta[s * C::NDB + b], op[s], acc[b]);
    op[0] = opn[0];
    op[1] = opn[1];
  };
  int t = 0;
  for (; t + W::RSLOT <= nt; t += W::RSLOT) {
    static_for<W::RSLOT>([&](auto J) {
      constexpr int j = decltype(J)::value;
      step(t + j, (j + 1) % W::RSLOT, (j + W::RSLOT - 1) % W::RSLOT);
    });
  }
  for (; t < nt; ++t) step(t, (t + 1) % W::RSLOT, (t + W::RSLOT - 1) % W::RSLOT);
  vmcnt_wait_all();
  if (!active) return;
#if QA_DQW_TR8
  const long r = (long)bh * Sq + q0 + 8 * ((c32 & 15) >> 2) + 4 * (c32 >> 4) + (c32 & 3);
#else
  const long r = (long)bh * Sq + q0 + c32;
#endif
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4h w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (_Float16)(acc[b][4 * g + j] * sms);
      *reinterpret_cast<v4h*>(dq + r * D + 32 * b + 8 * g + 4 * h) = w;
    }
  }
}

}  // namespace qattn

using namespace qattn;

// dO_i8 / s_dO (per 32-row block, int8:372-374), optional bf16 image of dO_i8, LD = {lse, D} per row.
extern "C" int qattn_int8_bwd_prep(const void* dO, const void* O, const void* lse, void* dO_i8,
                                   void* sdO, void* LD, void* dO_bf, long bh, long seq, int head_dim,
                                   void* stream) {
  if (seq % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  const long nblocks = bh * seq / 32;
  if (nblocks == 0) return 0;
  dim3 grid((unsigned)((nblocks + 3) / 4)), block(256);
  hipStream_t st = (hipStream_t)stream;
#define QA_LAUNCH(Dv, IM)                                                                       \
  hipLaunchKernelGGL((int8_bwd_prep_kernel<Dv, IM>), grid, block, 0, st, (const _Float16*)dO,   \
                     (const _Float16*)O, (const _Float16*)lse, (int8_t*)dO_i8, (_Float16*)sdO,   \
                     (__bf16*)dO_bf, (float2*)LD, nblocks)
  if (head_dim == 128) {
    if (dO_bf) QA_LAUNCH(128, true); else QA_LAUNCH(128, false);
  } else {
    if (dO_bf) QA_LAUNCH(64, true); else QA_LAUNCH(64, false);
  }
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_i8_to_bf16(const void* x, void* y, long n, void* stream) {
  if (n % 16 != 0) return 1;
  const long n16 = n / 16;
  if (n16 == 0) return 0;
  hipLaunchKernelGGL(i8_to_bf16_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const int8_t*)x, (__bf16*)y, n16);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

template <int D, int ROLE, bool CAUSAL, bool WS>
static void launch_bwd_c(const void* x8a, const void* x8b, const void* sxa, const void* sxb,
                         const void* y8a, const void* y8b, const void* ytr, const void* ytr2,
                         const void* yld, const void* sya, const void* syb, const void* xld, void* out,
                         void* out2, long bhx, long sx, long ny, int ydiv, long smod, float qks,
                         float sms, void* ds8, void* sds, hipStream_t st) {
  using G = BwdCfg<D, ROLE>;
  const int lds = G::NSLOT * G::SLOT + (int)((2 * (ny / 32) * 2 + 15) / 16 * 16) +
                  (WS ? G::WAVES * (int)(ny / 32) * 4 : 0);
  { static LdsGrant granted_; lds_grant((const void*)int8_bwd_kernel<D, ROLE, CAUSAL, WS>, lds, granted_); }
  const int nb = (int)((sx + G::XROWS - 1) / G::XROWS);
  hipLaunchKernelGGL((int8_bwd_kernel<D, ROLE, CAUSAL, WS>), dim3((unsigned)(nb * bhx)),
                     dim3(64 * G::WAVES), lds, st, (const int8_t*)x8a, (const int8_t*)x8b,
                     (const _Float16*)sxa, (const _Float16*)sxb, (const int8_t*)y8a,
                     (const int8_t*)y8b, (const __bf16*)ytr, (const __bf16*)ytr2, (const float2*)yld,
                     (const _Float16*)sya, (const _Float16*)syb, (const float2*)xld, (_Float16*)out,
                     (_Float16*)out2, (int)bhx, (int)sx, (int)ny, ydiv, (int)smod, qks, sms,
                     (int8_t*)ds8, (float*)sds);
}
template <int D, int ROLE, bool WS = false>
static void launch_bwd(int causal, const void* x8a, const void* x8b, const void* sxa, const void* sxb,
                       const void* y8a, const void* y8b, const void* ytr, const void* ytr2,
                       const void* yld, const void* sya, const void* syb, const void* xld, void* out,
                       void* out2, long bhx, long sx, long ny, int ydiv, long smod, float qks,
                       float sms, hipStream_t st, void* ds8 = nullptr, void* sds = nullptr) {
  if (causal)
    launch_bwd_c<D, ROLE, true, WS>(x8a, x8b, sxa, sxb, y8a, y8b, ytr, ytr2, yld, sya, syb, xld, out,
                                    out2, bhx, sx, ny, ydiv, smod, qks, sms, ds8, sds, st);
  else
    launch_bwd_c<D, ROLE, false, WS>(x8a, x8b, sxa, sxb, y8a, y8b, ytr, ytr2, yld, sya, syb, xld, out,
                                     out2, bhx, sx, ny, ydiv, smod, qks, sms, ds8, sds, st);
}

template <int D, bool CAUSAL>
static void launch_dqw_c(const void* ds8, const void* sds, const void* k_bf, const void* sk, void* dq,
                         long bh, long sqt, long skt, int group, float sms, hipStream_t st) {
  using G = DqwCfg<D>;
  const int nkt = (int)(skt / 32);
  const int lds = G::RBASE + G::RSLOT * G::REC + G::WAVES * nkt * 4 + 16;
  { static LdsGrant granted_; lds_grant((const void*)int8_bwd_dqw_kernel<D, CAUSAL>, lds, granted_); }
  const int nb = (int)((sqt + 32 * G::WAVES - 1) / (32 * G::WAVES));
  hipLaunchKernelGGL((int8_bwd_dqw_kernel<D, CAUSAL>), dim3((unsigned)(nb * bh)), dim3(64 * G::WAVES),
                     lds, st, (const int8_t*)ds8, (const float*)sds, (const __bf16*)k_bf,
                     (const _Float16*)sk, (_Float16*)dq, (int)bh, (int)sqt, (int)skt, group, sms);
}

// which: bit mask 1 = dV kernel, 4 = dK kernel, 8 = fused dK+dV kernel, 2 = dQ kernel,
// 16 = fused dK+dV kernel writing the dS workspace ws, 32 = dQ from the dS workspace.
// bh = batch * query heads; the key/value side has bh / group heads of skt rows.
template <int D>
static void bwd_launch_d(int which, const void* dO_i8, const void* sdO, const void* q_i8,
                         const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                         const void* sv, const void* LD, const void* q_bf, const void* k_bf,
                         const void* dO_bf, void* dq, void* dk, void* dv, long bh, long sqt, long skt,
                         int group, int causal, float qks, float sms, hipStream_t st,
                         void* ws = nullptr) {
  const long bkv = bh / group, ny = group * sqt;
  char* ds8 = (char*)ws;
  char* sds = ws ? ds8 + bh * (sqt / 32) * (skt / 32) * 1024 : nullptr;
  if (which & 16)
    launch_bwd<D, ROLE_DKV, true>(causal, k_i8, v_i8, sk, sv, q_i8, dO_i8, q_bf, dO_bf, LD, sq, sdO,
                                  nullptr, dk, dv, bkv, skt, ny, 1, sqt, qks, sms, st, ds8, sds);
  if (which & 32) {
    if (causal) launch_dqw_c<D, true>(ds8, sds, k_bf, sk, dq, bh, sqt, skt, group, sms, st);
    else launch_dqw_c<D, false>(ds8, sds, k_bf, sk, dq, bh, sqt, skt, group, sms, st);
  }
  // dV: own K (x8a) / streamed Q8 (y8a), dO image (ytr), LD; scales: sk|sv own, sq|sdO streamed
  if (which & 1)
    launch_bwd<D, ROLE_DV>(causal, k_i8, nullptr, sk, sv, q_i8, nullptr, dO_bf, nullptr, LD, sq, sdO,
                           nullptr, dv, nullptr, bkv, skt, ny, 1, sqt, qks, sms, st);
  // dK: own K, V / streamed Q8, dO8, q image, LD
  if (which & 4)
    launch_bwd<D, ROLE_DK>(causal, k_i8, v_i8, sk, sv, q_i8, dO_i8, q_bf, nullptr, LD, sq, sdO, nullptr,
                           dk, nullptr, bkv, skt, ny, 1, sqt, qks, sms, st);
  // dK and dV in one pass: + dO image
  if (which & 8)
    launch_bwd<D, ROLE_DKV>(causal, k_i8, v_i8, sk, sv, q_i8, dO_i8, q_bf, dO_bf, LD, sq, sdO, nullptr,
                            dk, dv, bkv, skt, ny, 1, sqt, qks, sms, st);
  // dQ: own Q, dO (+ their LD row stats) / streamed K8, V8, k image; scales: sq|sdO own, sk|sv
  if (which & 2)
    launch_bwd<D, ROLE_DQ>(causal, q_i8, dO_i8, sq, sdO, k_i8, v_i8, k_bf, nullptr, nullptr, sk, sv, LD,
                           dq, nullptr, bh, sqt, skt, group, skt, qks, sms, st);
}

static int int8_bwd_launch(int which, const void* dO_i8, const void* sdO, const void* q_i8,
                           const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                           const void* sv, const void* LD, const void* q_bf, const void* k_bf,
                           const void* dO_bf, void* dq, void* dk, void* dv, long bh, long sqt,
                           long skt, int group, int causal, int head_dim, float qks, float sms,
                           void* stream, void* ws = nullptr) {
  if (sqt % 32 != 0 || skt % 32 != 0 || group < 1 || bh % group != 0 ||
      (head_dim != 64 && head_dim != 128))
    return 1;
  if (bh == 0 || sqt == 0 || skt == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    bwd_launch_d<128>(which, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, k_bf, dO_bf, dq, dk,
                      dv, bh, sqt, skt, group, causal, qks, sms, st, ws);
  else
    bwd_launch_d<64>(which, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, k_bf, dO_bf, dq, dk,
                     dv, bh, sqt, skt, group, causal, qks, sms, st, ws);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_attn_bwd_ex(const void* dO_i8, const void* sdO, const void* q_i8,
                                      const void* sq, const void* k_i8, const void* sk,
                                      const void* v_i8, const void* sv, const void* LD,
                                      const void* q_bf, const void* k_bf, const void* dO_bf, void* dq,
                                      void* dk, void* dv, long bh, long sq_tok, long sk_tok, int group,
                                      int causal, int head_dim, float qks, float sms, void* stream) {
  return int8_bwd_launch(8 | 2, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, k_bf, dO_bf, dq, dk,
                         dv, bh, sq_tok, sk_tok, group, causal, head_dim, qks, sms, stream);
}

extern "C" int qattn_int8_attn_bwd(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* k_bf,
                                   const void* dO_bf, void* dq, void* dk, void* dv, long bh, long seq,
                                   int head_dim, float qks, float sms, void* stream) {
  return int8_bwd_launch(8 | 2, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, k_bf, dO_bf, dq, dk,
                         dv, bh, seq, seq, 1, 0, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dkdv(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* dO_bf,
                                   void* dk, void* dv, long bh, long seq, int head_dim, float qks,
                                   float sms, void* stream) {
  return int8_bwd_launch(8, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, nullptr, dO_bf,
                         nullptr, dk, dv, bh, seq, seq, 1, 0, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dv(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* dO_bf,
                                   void* dk, void* dv, long bh, long seq, int head_dim, float qks,
                                   float sms, void* stream) {
  return int8_bwd_launch(1, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, nullptr, dO_bf,
                         nullptr, dk, dv, bh, seq, seq, 1, 0, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dk(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* dO_bf,
                                   void* dk, void* dv, long bh, long seq, int head_dim, float qks,
                                   float sms, void* stream) {
  return int8_bwd_launch(4, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, nullptr, dO_bf,
                         nullptr, dk, dv, bh, seq, seq, 1, 0, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dq(const void* dO_i8, const void* sdO, const void* q_i8,
                                 const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                 const void* sv, const void* LD, const void* k_bf, void* dq, long bh,
                                 long seq, int head_dim, float qks, float sms, void* stream) {
  return int8_bwd_launch(2, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, nullptr, k_bf, nullptr, dq,
                         nullptr, nullptr, bh, seq, seq, 1, 0, head_dim, qks, sms, stream);
}

// The dK+dV kernel addresses the records of one key/value head (its G query heads) with 32-bit
// buffer offsets: that region, G * (sq/32) * (sk/32) KiB, must stay below 2^31 bytes.
static bool ws_region_fits(long group, long sq_tok, long sk_tok) {
  return group * (sq_tok / 32) * (sk_tok / 32) * 1024 < (1L << 31);
}

// Largest dS-record workspace either backward (int8 or bf16) allocates before it falls back to
// recomputation: QATTN_BWD_WS_MAX bytes if set, else 16 GiB.  A fixed figure, not the device's free
// memory: hipMemGetInfo does not see what the caller's caching allocator holds reserved, so a free-
// memory cap would depend on allocator history; an allocation that fails falls back to the
// recomputing backward instead (same results).
extern "C" long qattn_bwd_ws_cap(void) {
  const char* s = getenv("QATTN_BWD_WS_MAX");
  if (s != nullptr && *s != 0) return strtol(s, nullptr, 10);
  return 16L << 30;
}

extern "C" long qattn_int8_bwd_ws_bytes(long bh, long sq_tok, long sk_tok) {
  if (sq_tok % 32 != 0 || sk_tok % 32 != 0 || bh < 0) return -1;
  if (!ws_region_fits(1, sq_tok, sk_tok)) return -1;   // too large even ungrouped: recompute instead
  return bh * (sq_tok / 32) * (sk_tok / 32) * (1024 + 4);
}

extern "C" int qattn_int8_attn_bwd_ws(const void* dO_i8, const void* sdO, const void* q_i8,
                                      const void* sq, const void* k_i8, const void* sk,
                                      const void* v_i8, const void* sv, const void* LD,
                                      const void* q_bf, const void* k_bf, const void* dO_bf, void* dq,
                                      void* dk, void* dv, void* ws, long bh, long sq_tok, long sk_tok,
                                      int group, int causal, int head_dim, float qks, float sms,
                                      void* stream) {
  if (ws == nullptr || group < 1 || !ws_region_fits(group, sq_tok, sk_tok)) return 1;
  return int8_bwd_launch(16 | 32, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD,
                         q_bf, k_bf, dO_bf, dq, dk, dv, bh, sq_tok, sk_tok, group, causal, head_dim, qks,
                         sms, stream, ws);
}

// qattn_int8_attn_bwd_ws over chunks of kv_chunk key/value heads (with their group query heads):
// dK+dV of a chunk writes its records into ws, the dQ pass of the same chunk reads them, and the next
// chunk re-uses the same ws bytes.  Every tensor is head-major and contiguous, so a chunk is a plain
// pointer offset; results are bit-identical to the one-shot call (each head's arithmetic is
// unchanged).  The chunk size is the caller's: a chunk's records stay in the 256 MB Infinity Cache
// between their write and their read only if the chunk's records plus the other bytes both passes
// move stay under ~256 MB (MI355X_MICROARCH "Infinity Cache"); the default chunk at config 3 (32
// heads, 539 MB of records) does not, so there the records go through HBM.  What chunking buys
// there is a quarter of the workspace and a measured 2-4 % (attention_int8.WS_CHUNK).
extern "C" int qattn_int8_attn_bwd_wsc(const void* dO_i8, const void* sdO, const void* q_i8,
                                       const void* sq, const void* k_i8, const void* sk,
                                       const void* v_i8, const void* sv, const void* LD,
                                       const void* q_bf, const void* k_bf, const void* dO_bf, void* dq,
                                       void* dk, void* dv, void* ws, long kv_chunk, long bh,
                                       long sq_tok, long sk_tok, int group, int causal, int head_dim,
                                       float qks, float sms, void* stream) {
  if (ws == nullptr || group < 1 || kv_chunk < 1 || !ws_region_fits(group, sq_tok, sk_tok)) return 1;
  if (sq_tok % 32 != 0 || sk_tok % 32 != 0 || bh % group != 0 || (head_dim != 64 && head_dim != 128))
    return 1;
  const long bkv = bh / group, D = head_dim;
  auto at = [](const void* p, long bytes) { return (void*)((const char*)p + bytes); };
  for (long k0 = 0; k0 < bkv; k0 += kv_chunk) {
    const long nkv = std::min(kv_chunk, bkv - k0);
    const long qr = k0 * group * sq_tok, kr = k0 * sk_tok;   // first query / key row of the chunk
    const int rc = int8_bwd_launch(
        16 | 32, at(dO_i8, qr * D), at(sdO, qr / 32 * 2), at(q_i8, qr * D), at(sq, qr / 32 * 2),
        at(k_i8, kr * D), at(sk, kr / 32 * 2), at(v_i8, kr * D), at(sv, kr / 32 * 2), at(LD, qr * 8),
        at(q_bf, qr * D * 2), at(k_bf, kr * D * 2), at(dO_bf, qr * D * 2), at(dq, qr * D * 2),
        at(dk, kr * D * 2), at(dv, kr * D * 2), nkv * group, sq_tok, sk_tok, group, causal, head_dim,
        qks, sms, stream, ws);
    if (rc != 0) return rc;
  }
  return 0;
}

#if QA_DKV_STAMP
extern "C" int qattn_dkv_stamps(void* host_dst) {
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(qattn::g_dkv_stamp), sizeof(qattn::g_dkv_stamp)) == hipSuccess ? 0 : 2;
}
#endif

// The two parts of qattn_int8_attn_bwd_ws, launchable alone (per-kernel timing).
extern "C" int qattn_int8_bwd_dkdv_ws(const void* dO_i8, const void* sdO, const void* q_i8,
                                      const void* sq, const void* k_i8, const void* sk,
                                      const void* v_i8, const void* sv, const void* LD,
                                      const void* q_bf, const void* dO_bf, void* dk, void* dv, void* ws,
                                      long bh, long seq, int head_dim, float qks, float sms,
                                      void* stream) {
  if (ws == nullptr || !ws_region_fits(1, seq, seq)) return 1;
  return int8_bwd_launch(16, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf,
                         nullptr, dO_bf, nullptr, dk, dv, bh, seq, seq, 1, 0, head_dim, qks, sms, stream,
                         ws);
}
extern "C" int qattn_int8_bwd_dq_ws(const void* k_bf, const void* sk, void* dq, void* ws, long bh,
                                    long seq, int head_dim, float sms, void* stream) {
  if (ws == nullptr) return 1;
  return int8_bwd_launch(32, nullptr, nullptr, nullptr, nullptr, nullptr, sk, nullptr, nullptr,
                         nullptr, nullptr, k_bf, nullptr, dq, nullptr, nullptr, bh, seq, seq, 1, 0,
                         head_dim, 0.f, sms, stream, ws);
}
