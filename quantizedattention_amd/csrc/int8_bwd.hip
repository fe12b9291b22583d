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
#include "common.h"

namespace qattn {

template <int D>
struct I8BwdCfg {
  static constexpr int NKS8 = D / 32;    // i8 k-steps over D
  static constexpr int NDB = D / 32;
  static constexpr int T8 = 32 * D;      // 32-row int8 tile bytes
  static constexpr int T16 = 64 * D;     // 32-row bf16 tile bytes
  // kernel A stage: Q8, O8 (int8 rows), QB, OB (bf16 tr), LD (32 x {lse, D} f32)
  static constexpr int A_STAGE = 2 * T8 + 2 * T16 + 256;
  static constexpr int A_INST = (2 * T8 + 2 * T16) / 1024 + 1;   // + 1 dword-DMA for LD
  static constexpr int A_IPW = (A_INST + 3) / 4;                  // per wave (padded)
  // kernel A split by output (MODE 1 = dV only: Q8, OB, LD; MODE 2 = dK only: Q8, O8, QB, LD)
  static constexpr int A1_STAGE = T8 + T16 + 256;
  static constexpr int A1_IPW = ((T8 + T16) / 1024 + 1 + 3) / 4;
  static constexpr int A2_STAGE = 2 * T8 + T16 + 256;
  static constexpr int A2_IPW = ((2 * T8 + T16) / 1024 + 1 + 3) / 4;
  // kernel B stage: K8, V8 (int8 rows), KB (bf16 tr)
  static constexpr int B_STAGE = 2 * T8 + T16;
  static constexpr int B_INST = B_STAGE / 1024;
  static constexpr int B_IPW = B_INST / 4;
};
template <int D>
QA_DEVICE int i8_sw(int row) { return (row >> ((D == 128) ? 1 : 2)) & (D / 16 - 1); }
template <int D>
QA_DEVICE int t16_sw(int row) { return (row & 3) << ((D == 128) ? 2 : 1); }

// Global chunk that lands at LDS position (row, p) of a swizzled image with `nch` 16-B chunks/row.
template <int D, bool TR>
QA_DEVICE int src_chunk(int row, int p) { return p ^ (TR ? t16_sw<D>(row) : i8_sw<D>(row)); }

// LDS-DMA of instruction `inst` (1 KiB) of a 32-row tile: rows of RB bytes at gsrc (row stride RB).
template <int D, int RB, bool TR>
QA_DEVICE void dma_tile_inst(const char* gsrc, char* lds_tile, int inst, int lane) {
  constexpr int NCH = RB / 16, RPI = 64 / NCH;
  const int row = inst * RPI + lane / NCH, p = lane % NCH;
  glds16(gsrc + (long)row * RB + 16 * src_chunk<D, TR>(row, p), lds_tile + inst * 1024);
}
// dword LDS-DMA (64 lanes x 4 B = 256 B, lane-linear)
QA_DEVICE void glds4(const void* gsrc, void* lds_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)(lds_base));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}
template <int N>
QA_DEVICE void vmcnt_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// A operand (X^T, 32 d x 16 rows) of a 32x32x16 product from a bf16 [row][d] tr image.
template <int D>
QA_DEVICE v8bf t16_frag(const char* base, int row_base, int b, int lane) {
  const int h = lane >> 5, gg = (lane >> 4) & 1, i16 = lane & 15;
  const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
  const int row = row_base + 4 * h + (i16 >> 2);
  const int ch = d / 8, within = (d % 8) * 2;
  return __builtin_bit_cast(
      v8bf, ds_read_tr16_x2(base + row * 2 * D + 16 * (ch ^ t16_sw<D>(row)) + within,
                            base + (row + 8) * 2 * D + 16 * (ch ^ t16_sw<D>(row + 8)) + within));
}
QA_DEVICE float max16_abs(const float* x) {
  float m0 = vmax(fabsf(x[0]), fabsf(x[1])), m1 = vmax(fabsf(x[2]), fabsf(x[3]));
  float m2 = vmax(fabsf(x[4]), fabsf(x[5])), m3 = vmax(fabsf(x[6]), fabsf(x[7]));
  float m4 = vmax(fabsf(x[8]), fabsf(x[9])), m5 = vmax(fabsf(x[10]), fabsf(x[11]));
  float m6 = vmax(fabsf(x[12]), fabsf(x[13])), m7 = vmax(fabsf(x[14]), fabsf(x[15]));
  return vmax(vmax(vmax(m0, m1), vmax(m2, m3)), vmax(vmax(m4, m5), vmax(m6, m7)));
}
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
// LD[row] = {fp32(lse[row]), fp16(sum_d fp32(fp16(dO*O)))} (int8:360, int8:398)
template <int D>
__global__ __launch_bounds__(256) void int8_bwd_ld_kernel(const _Float16* __restrict__ dO,
                                                          const _Float16* __restrict__ O,
                                                          const _Float16* __restrict__ lse,
                                                          float2* __restrict__ LD, long rows) {
  constexpr int LPR = D / 8;
  const long row = ((long)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int c = (threadIdx.x % LPR) * 8;
  float acc = 0.f;
  if (row < rows) {
    const v8h a = *reinterpret_cast<const v8h*>(dO + row * D + c);
    const v8h b = *reinterpret_cast<const v8h*>(O + row * D + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (float)(_Float16)((float)a[j] * (float)b[j]);
  }
#pragma unroll
  for (int o = LPR / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if (row < rows && (threadIdx.x % LPR) == 0) LD[row] = float2{(float)lse[row], (float)(_Float16)acc};
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

// ------------------------------------------------------------------------- kernel A: dK, dV
// MODE 0: dK and dV in one pass (1 wave/SIMD: 2 x 64 fp32 accumulator registers);
// MODE 1: dV only (S -> P -> P_i8 operand);  MODE 2: dK only (S, dP -> dS -> dS_i8 operand).
// The split pair re-computes S (4 extra int8 MFMAs per tile) but halves the accumulator registers,
// so each kernel runs at 2-3 waves per SIMD.
template <int D, int MODE>
struct AStage {
  using C = I8BwdCfg<D>;
  static constexpr bool NEED_O8 = MODE != 1, NEED_QB = MODE != 1, NEED_OB = MODE != 2;
  static constexpr int Q8 = 0;
  static constexpr int O8 = Q8 + C::T8;
  static constexpr int QB = O8 + (NEED_O8 ? C::T8 : 0);
  static constexpr int OB = QB + (NEED_QB ? C::T16 : 0);
  static constexpr int LDO = OB + (NEED_OB ? C::T16 : 0);
  static constexpr int BYTES = LDO + 256;
  static constexpr int N8 = C::T8 / 1024, N16 = C::T16 / 1024;
  static constexpr int INST = N8 + (NEED_O8 ? N8 : 0) + (NEED_QB ? N16 : 0) + (NEED_OB ? N16 : 0) + 1;
  static constexpr int IPW = (INST + 3) / 4;
};

template <int D, int MODE>
__global__ __launch_bounds__(256, MODE == 0 ? 1 : 2) void int8_bwd_dkdv_kernel(
    const int8_t* __restrict__ dOi, const _Float16* __restrict__ sdO, const int8_t* __restrict__ qi,
    const _Float16* __restrict__ sq, const int8_t* __restrict__ ki, const _Float16* __restrict__ sk,
    const int8_t* __restrict__ vi, const _Float16* __restrict__ sv, const float2* __restrict__ LD,
    const __bf16* __restrict__ qb, const __bf16* __restrict__ ob, _Float16* __restrict__ dk,
    _Float16* __restrict__ dv, int BH, int S, float qks, float sms) {
  using C = I8BwdCfg<D>;
  using G = AStage<D, MODE>;
  constexpr bool DO_DV = MODE != 2, DO_DK = MODE != 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nkb = (S + 127) / 128;
  int bh, kt;
  xcd_remap(blockIdx.x, nkb, BH, bh, kt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int k0 = kt * 128 + wave * 32;
  const bool active = k0 < S;
  const long hrow = (long)bh * S;
  const int nqt = S / 32;

  // one q-tile stage: wave w issues DMA slots w, w+4, ...; slots past the real instructions repeat
  // the LD dword DMA (same bytes, benign) so that every wave issues exactly G::IPW (counted vmcnt).
  auto stage = [&](int t, int buf) {
    t = min(t, nqt - 1);
    const long r0 = hrow + 32L * t;
    char* base = smem + buf * G::BYTES;
    for (int i = 0; i < G::IPW; ++i) {
      int inst = wave + 4 * i;
      if (inst < G::N8) {
        dma_tile_inst<D, D, false>(reinterpret_cast<const char*>(qi + r0 * D), base + G::Q8, inst, lane);
        continue;
      }
      inst -= G::N8;
      if constexpr (G::NEED_O8) {
        if (inst < G::N8) {
          dma_tile_inst<D, D, false>(reinterpret_cast<const char*>(dOi + r0 * D), base + G::O8, inst, lane);
          continue;
        }
        inst -= G::N8;
      }
      if constexpr (G::NEED_QB) {
        if (inst < G::N16) {
          dma_tile_inst<D, 2 * D, true>(reinterpret_cast<const char*>(qb + r0 * D), base + G::QB, inst, lane);
          continue;
        }
        inst -= G::N16;
      }
      if constexpr (G::NEED_OB) {
        if (inst < G::N16) {
          dma_tile_inst<D, 2 * D, true>(reinterpret_cast<const char*>(ob + r0 * D), base + G::OB, inst, lane);
          continue;
        }
      }
      glds4(reinterpret_cast<const char*>(LD + r0) + 4 * lane, base + G::LDO);
    }
  };
  stage(0, 0);
  stage(1, 1);
  // per-tile q / dO scales of the head, once, in LDS (a vector global load inside the loop would
  // make hipcc wait vmcnt for the in-flight LDS-DMA)
  _Float16* sc_lds = reinterpret_cast<_Float16*>(smem + 3 * G::BYTES);
  for (int i = tid; i < nqt; i += 256) {
    sc_lds[i] = sq[hrow / 32 + i];
    sc_lds[nqt + i] = sdO[hrow / 32 + i];
  }

  v4i kfr[C::NKS8], vfr[C::NKS8];
  float skw = 0.f, svw = 0.f;
  if (active) {
    const int8_t* kr = ki + (hrow + k0 + c32) * D + 16 * h;
    const int8_t* vr = vi + (hrow + k0 + c32) * D + 16 * h;
#pragma unroll
    for (int s = 0; s < C::NKS8; ++s) {
      kfr[s] = *reinterpret_cast<const v4i*>(kr + 32 * s);
      if constexpr (DO_DK) vfr[s] = *reinterpret_cast<const v4i*>(vr + 32 * s);
    }
    skw = (float)sk[(hrow + k0) / 32];
    svw = (float)sv[(hrow + k0) / 32];
  }
  const float ck = skw * qks;
  v16f dka[C::NDB], dva[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) { dka[b] = v16f{}; dva[b] = v16f{}; }
  int roff[C::NKS8];
#pragma unroll
  for (int s = 0; s < C::NKS8; ++s) roff[s] = c32 * D + 16 * ((2 * s + h) ^ i8_sw<D>(c32));

  vmem_drain();
  vmcnt_wait<0>();
  __syncthreads();
  for (int t = 0; t < nqt; ++t) {
    const int buf = t % 3;
    stage(t + 2, (t + 2) % 3);
    const char* base = smem + buf * G::BYTES;
    const float* ld = reinterpret_cast<const float*>(base + G::LDO);
    const float sqt = (float)sc_lds[t];
    const float sdt = (float)sc_lds[nqt + t];
    if (active) {
      v16i sacc = v16i{}, pacc = v16i{};
#pragma unroll
      for (int s = 0; s < C::NKS8; ++s) {
        sacc = mfma_i8(*reinterpret_cast<const v4i*>(base + G::Q8 + roff[s]), kfr[s], sacc);
        if constexpr (DO_DK)
          pacc = mfma_i8(*reinterpret_cast<const v4i*>(base + G::O8 + roff[s]), vfr[s], pacc);
      }
      const float c1 = sqt * ck, c2 = sdt * svw;
      float P[16], dS[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f a = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h));
        const v4f b = *reinterpret_cast<const v4f*>(ld + 2 * (8 * g + 4 * h) + 4);
        const float lse_r[4] = {a[0], a[2], b[0], b[2]};
        const float d_r[4] = {a[1], a[3], b[1], b[3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g + j;
          P[i] = exp2_f32(fmaf((float)sacc[i], c1, -lse_r[j]));
          if constexpr (DO_DK) dS[i] = P[i] * fmaf((float)pacc[i], c2, -d_r[j]);
        }
      }
      if constexpr (DO_DV) {
        const float pmax = wave_max_dpp(max16_abs(P));
        const float sP = pmax * (1.0f / 127.0f);
        v8bf pb[2];
        quant_operand(P, sP > 0.f ? 127.0f / pmax : 0.f, sP * sdt, pb);
#pragma unroll
        for (int b = 0; b < C::NDB; ++b)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            dva[b] = mfma_bf16(t16_frag<D>(base + G::OB, 16 * s, b, lane), pb[s], dva[b]);
      }
      if constexpr (DO_DK) {
        const float smax = wave_max_dpp(max16_abs(dS));
        const float ssd = smax * (1.0f / 127.0f);
        v8bf sb[2];
        quant_operand(dS, ssd > 0.f ? 127.0f / smax : 0.f, ssd * sqt, sb);
#pragma unroll
        for (int b = 0; b < C::NDB; ++b)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            dka[b] = mfma_bf16(t16_frag<D>(base + G::QB, 16 * s, b, lane), sb[s], dka[b]);
      }
    }
    vmcnt_wait<G::IPW>();   // tile t+1 (issued last iteration) has landed; t+2 may be in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  vmcnt_wait<0>();
  if (!active) return;
  const long krow = hrow + k0 + c32;
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4h wk, wv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        wk[j] = (_Float16)(dka[b][4 * g + j] * sms);
        wv[j] = (_Float16)dva[b][4 * g + j];
      }
      if constexpr (DO_DK) *reinterpret_cast<v4h*>(dk + krow * D + 32 * b + 8 * g + 4 * h) = wk;
      if constexpr (DO_DV) *reinterpret_cast<v4h*>(dv + krow * D + 32 * b + 8 * g + 4 * h) = wv;
    }
  }
}

// ----------------------------------------------------------------------------- kernel B: dQ
template <int D>
__global__ __launch_bounds__(256, 2) void int8_bwd_dq_kernel(
    const int8_t* __restrict__ dOi, const _Float16* __restrict__ sdO, const int8_t* __restrict__ qi,
    const _Float16* __restrict__ sq, const int8_t* __restrict__ ki, const _Float16* __restrict__ sk,
    const int8_t* __restrict__ vi, const _Float16* __restrict__ sv, const float2* __restrict__ LD,
    const __bf16* __restrict__ kb16, _Float16* __restrict__ dq, int BH, int S, float qks, float sms) {
  using C = I8BwdCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (S + 127) / 128;
  int bh, qt;
  xcd_remap(blockIdx.x, nqb, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qt * 128 + wave * 32;
  const bool active = q0 < S;
  const long hrow = (long)bh * S;
  const int nkt = S / 32;

  auto stage = [&](int t, int buf) {
    t = min(t, nkt - 1);
    const long r0 = hrow + 32L * t;
    char* base = smem + buf * C::B_STAGE;
    for (int i = 0; i < C::B_IPW; ++i) {
      int inst = wave + 4 * i;
      constexpr int n8 = C::T8 / 1024;
      if (inst < n8) {
        dma_tile_inst<D, D, false>(reinterpret_cast<const char*>(ki + r0 * D), base, inst, lane);
      } else if ((inst -= n8) < n8) {
        dma_tile_inst<D, D, false>(reinterpret_cast<const char*>(vi + r0 * D), base + C::T8, inst, lane);
      } else {
        inst -= n8;
        dma_tile_inst<D, 2 * D, true>(reinterpret_cast<const char*>(kb16 + r0 * D), base + 2 * C::T8,
                                      inst, lane);
      }
    }
  };
  stage(0, 0);
  stage(1, 1);
  _Float16* sc_lds = reinterpret_cast<_Float16*>(smem + 3 * C::B_STAGE);
  for (int i = tid; i < nkt; i += 256) {
    sc_lds[i] = sk[hrow / 32 + i];
    sc_lds[nkt + i] = sv[hrow / 32 + i];
  }

  v4i qfr[C::NKS8], ofr[C::NKS8];
  float lq = 0.f, Dq = 0.f, sqw = 0.f, sdw = 0.f;
  if (active) {
    const long r = hrow + q0 + c32;
#pragma unroll
    for (int s = 0; s < C::NKS8; ++s) {
      qfr[s] = *reinterpret_cast<const v4i*>(qi + r * D + 16 * h + 32 * s);
      ofr[s] = *reinterpret_cast<const v4i*>(dOi + r * D + 16 * h + 32 * s);
    }
    const float2 ldr = LD[r];
    lq = ldr.x;
    Dq = ldr.y;
    sqw = (float)sq[(hrow + q0) / 32];
    sdw = (float)sdO[(hrow + q0) / 32];
  }
  const float cq = sqw * qks;
  v16f acc[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) acc[b] = v16f{};
  int roff[C::NKS8];
#pragma unroll
  for (int s = 0; s < C::NKS8; ++s) roff[s] = c32 * D + 16 * ((2 * s + h) ^ i8_sw<D>(c32));

  vmem_drain();
  vmcnt_wait<0>();
  __syncthreads();
  for (int t = 0; t < nkt; ++t) {
    const int buf = t % 3;
    stage(t + 2, (t + 2) % 3);
    const char* base = smem + buf * C::B_STAGE;
    const char* k8 = base;
    const char* v8 = base + C::T8;
    const char* kbl = base + 2 * C::T8;
    const float skt = (float)sc_lds[t];
    const float svt = (float)sc_lds[nkt + t];
    if (active) {
      v16i sacc = v16i{}, pacc = v16i{};
#pragma unroll
      for (int s = 0; s < C::NKS8; ++s) {
        sacc = mfma_i8(*reinterpret_cast<const v4i*>(k8 + roff[s]), qfr[s], sacc);
        pacc = mfma_i8(*reinterpret_cast<const v4i*>(v8 + roff[s]), ofr[s], pacc);
      }
      // same per-element operation order as kernel A:  ((acc*sq)*sk*qks) -> fma with -lse
      const float c1 = sqw * (skt * qks), c2 = sdw * svt;
      float dS[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float P = exp2_f32(fmaf((float)sacc[i], c1, -lq));
        dS[i] = P * fmaf((float)pacc[i], c2, -Dq);
      }
      const float smax = wave_max_dpp(max16_abs(dS));
      const float ssd = smax * (1.0f / 127.0f);
      v8bf sb[2];
      quant_operand(dS, ssd > 0.f ? 127.0f / smax : 0.f, ssd * skt, sb);
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
        for (int s = 0; s < 2; ++s) acc[b] = mfma_bf16(t16_frag<D>(kbl, 16 * s, b, lane), sb[s], acc[b]);
      }
    }
    vmcnt_wait<C::B_IPW>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  vmcnt_wait<0>();
  (void)cq;
  if (!active) return;
  const long r = hrow + q0 + c32;
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

extern "C" int qattn_int8_quant(const void* x, void* idx, void* scale, void* deq, const void* kmean,
                                long rows, int rows_per_head, int head_dim, void* stream);

// dO_i8 / s_dO (per 32-row block, int8:372-374) and LD = {lse, D} per row.
extern "C" int qattn_int8_bwd_prep(const void* dO, const void* O, const void* lse, void* dO_i8,
                                   void* sdO, void* LD, long bh, long seq, int head_dim, void* stream) {
  if (seq % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  const long rows = bh * seq;
  if (rows == 0) return 0;
  int rc = qattn_int8_quant(dO, dO_i8, sdO, nullptr, nullptr, rows, (int)seq, head_dim, stream);
  if (rc) return rc;
  const int rpb = 256 / (head_dim / 8);
  dim3 grid((unsigned)((rows + rpb - 1) / rpb)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL((int8_bwd_ld_kernel<128>), grid, block, 0, st, (const _Float16*)dO,
                       (const _Float16*)O, (const _Float16*)lse, (float2*)LD, rows);
  else
    hipLaunchKernelGGL((int8_bwd_ld_kernel<64>), grid, block, 0, st, (const _Float16*)dO,
                       (const _Float16*)O, (const _Float16*)lse, (float2*)LD, rows);
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

// which: 1 = dK/dV kernel, 2 = dQ kernel, 3 = both
static int int8_bwd_launch(int which, const void* dO_i8, const void* sdO, const void* q_i8,
                           const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                           const void* sv, const void* LD, const void* q_bf, const void* k_bf,
                           const void* dO_bf, void* dq, void* dk, void* dv, long bh, long seq,
                           int head_dim, float qks, float sms, void* stream) {
  if (seq % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0 || seq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)((seq + 127) / 128);
#define QA_LAUNCH_A(Dv, M)                                                                       \
  {                                                                                              \
    const int sA = 3 * AStage<Dv, M>::BYTES + sc;                                                \
    hipFuncSetAttribute((const void*)int8_bwd_dkdv_kernel<Dv, M>,                                \
                        hipFuncAttributeMaxDynamicSharedMemorySize, sA);                         \
    hipLaunchKernelGGL((int8_bwd_dkdv_kernel<Dv, M>), dim3((unsigned)(nb * bh)), dim3(256), sA,   \
                       st, (const int8_t*)dO_i8, (const _Float16*)sdO, (const int8_t*)q_i8,       \
                       (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,             \
                       (const int8_t*)v_i8, (const _Float16*)sv, (const float2*)LD,               \
                       (const __bf16*)q_bf, (const __bf16*)dO_bf, (_Float16*)dk, (_Float16*)dv,    \
                       (int)bh, (int)seq, qks, sms);                                             \
  }
#define QA_LAUNCH(Dv)                                                                            \
  {                                                                                              \
    using C = I8BwdCfg<Dv>;                                                                      \
    const int sc = (int)((2 * (seq / 32) * 2 + 15) / 16 * 16);                                   \
    const int sB = 3 * C::B_STAGE + sc;                                                          \
    if (which & 1) QA_LAUNCH_A(Dv, 1)                                                            \
    if (which & 4) QA_LAUNCH_A(Dv, 2)                                                            \
    if (which & 2) {                                                                             \
      hipFuncSetAttribute((const void*)int8_bwd_dq_kernel<Dv>,                                   \
                          hipFuncAttributeMaxDynamicSharedMemorySize, sB);                       \
      hipLaunchKernelGGL((int8_bwd_dq_kernel<Dv>), dim3((unsigned)(nb * bh)), dim3(256), sB, st,  \
                         (const int8_t*)dO_i8, (const _Float16*)sdO, (const int8_t*)q_i8,         \
                         (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,           \
                         (const int8_t*)v_i8, (const _Float16*)sv, (const float2*)LD,             \
                         (const __bf16*)k_bf, (_Float16*)dq, (int)bh, (int)seq, qks, sms);        \
    }                                                                                            \
  }
  if (head_dim == 128) QA_LAUNCH(128) else QA_LAUNCH(64)
#undef QA_LAUNCH
#undef QA_LAUNCH_A
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_attn_bwd(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* k_bf,
                                   const void* dO_bf, void* dq, void* dk, void* dv, long bh, long seq,
                                   int head_dim, float qks, float sms, void* stream) {
  return int8_bwd_launch(7, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, k_bf, dO_bf, dq, dk,
                         dv, bh, seq, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dkdv(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* dO_bf,
                                   void* dk, void* dv, long bh, long seq, int head_dim, float qks,
                                   float sms, void* stream) {
  return int8_bwd_launch(5, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, nullptr, dO_bf,
                         nullptr, dk, dv, bh, seq, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dv(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* dO_bf,
                                   void* dk, void* dv, long bh, long seq, int head_dim, float qks,
                                   float sms, void* stream) {
  return int8_bwd_launch(1, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, nullptr, dO_bf,
                         nullptr, dk, dv, bh, seq, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dk(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* LD, const void* q_bf, const void* dO_bf,
                                   void* dk, void* dv, long bh, long seq, int head_dim, float qks,
                                   float sms, void* stream) {
  return int8_bwd_launch(4, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, nullptr, dO_bf,
                         nullptr, dk, dv, bh, seq, head_dim, qks, sms, stream);
}
extern "C" int qattn_int8_bwd_dq(const void* dO_i8, const void* sdO, const void* q_i8,
                                 const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                 const void* sv, const void* LD, const void* k_bf, void* dq, long bh,
                                 long seq, int head_dim, float qks, float sms, void* stream) {
  return int8_bwd_launch(2, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, nullptr, k_bf, nullptr, dq,
                         nullptr, nullptr, bh, seq, head_dim, qks, sms, stream);
}
