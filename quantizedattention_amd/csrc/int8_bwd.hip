// SageAttention-3 8-bit attention backward for gfx950; replaces helion_atten_int8_hl_dot_bwd
// (attention_int8.py:264-432) with the build-contract fixes of SURVEY F4, keeping the reference's
// quantisation recipe (per 32x32 (q-tile, k-tile) pair, Bq = Bkv = 32):
//   S   = fp16(((i32(q_i8 . k_i8) * sq) * sk) * qks)                  int8:352-355
//   P   = exp2(fp32(fp16(S - lse)))                                    int8:360
//   sP  = max(P) / 127 over the tile;  P_i8 = trunc(P / sP)           int8:363-365
//   dV += (P_i8^T . dO_i8) * s_dO * sP                                 int8:375-378 (F4: accumulate)
//   dP  = (i32(dO_i8 . v_i8) * s_dO) * sv ;  D = fp16(rowsum(fp16(dO*O)))   int8:382-398
//   dS  = P * (dP - D)                       (reference: S * (dP - D), F4)   int8:399
//   s_dS = max|dS| / 127 over the tile;  dS_i8 = trunc(dS / s_dS)    int8:403-405
//   dQ += (dS_i8 . k_i8) * s_dS * sk * sm_scale   (reference: qk_scale, racy fp16 RMW, k_mean term)
//   dK += (dS_i8^T . q_i8) * s_dS * sq * sm_scale (reference: overwrite per q-tile)
//
// S and dP (the two products whose dequantisation scale is uniform per 32x32 tile and which feed
// elementwise work anyway) run on v_mfma_i32_32x32x32_i8.  The three accumulating products fold
// their per-tile scalar into the quantised P / dS operand (bf16(P_i8 * sP * s_dO), bf16(dS_i8 *
// s_dS * sq|sk)) and multiply exact integer-valued bf16 copies of dO_i8 / q_i8 / k_i8 on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation: identical sums up to one bf16 rounding of the
// scaled operand, and no per-tile i32->f32 dequantisation of D-wide accumulators.
//
// Kernel A (dK, dV): workgroup = 4 waves x 32 keys, loops over query tiles (query rows in
// registers, key on the lane).  Kernel B (dQ): workgroup = 4 waves x 32 queries, loops over key
// tiles (keys in registers, query on the lane).  Both compute the (q-tile, k-tile) dS tile with
// the same operation order, so the tile scales and dS_i8 agree bit for bit.  No atomics.
#include "common.h"

namespace qattn {

template <int D>
struct I8BwdCfg {
  static constexpr int RB8 = D;          // bytes per int8 row
  static constexpr int NCH8 = D / 16;
  static constexpr int RB16 = 2 * D;     // bytes per bf16 row
  static constexpr int NCH16 = RB16 / 16;
  static constexpr int NKS8 = D / 32;    // i8 k-steps over D
  static constexpr int NDB = D / 32;
  static constexpr int T8 = 32 * RB8;    // 32-row int8 tile bytes
  static constexpr int T16 = 32 * RB16;  // 32-row bf16 tile bytes
};
// int8 row image (ds_read_b128 row reads)
template <int D>
QA_DEVICE int i8_off(int row, int ch) {
  constexpr int sh = (D == 128) ? 1 : 2;
  return row * D + 16 * (ch ^ ((row >> sh) & (D / 16 - 1)));
}
// bf16 transposed-read image (ds_read_b64_tr_b16)
template <int D>
QA_DEVICE int t16_off(int row, int ch) {
  constexpr int sh = (D == 128) ? 2 : 1;
  return row * 2 * D + 16 * (ch ^ ((row & 3) << sh));
}
template <int D>
QA_DEVICE v8bf t16_frag(const char* base, int row_base, int b, int lane) {
  const int h = lane >> 5, gg = (lane >> 4) & 1, i16 = lane & 15;
  const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
  const int row = row_base + 4 * h + (i16 >> 2);
  const int ch = d / 8, within = (d % 8) * 2;
  return __builtin_bit_cast(
      v8bf, ds_read_tr16_x2(base + t16_off<D>(row, ch) + within, base + t16_off<D>(row + 8, ch) + within));
}
// 16 int8 -> 16 exact bf16 (as two 16-B chunks)
QA_DEVICE void i8x16_to_bf16(v4i x, v4u& lo, v4u& hi) {
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int word = x[w];
    unsigned p[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float a = (float)((word << (24 - 16 * j)) >> 24);
      const float b = (float)((word << (16 - 16 * j)) >> 24);
      p[j] = (__float_as_uint(a) >> 16) | (__float_as_uint(b) & 0xffff0000u);
    }
    if (w < 2) { lo[2 * w] = p[0]; lo[2 * w + 1] = p[1]; }
    else { hi[2 * w - 4] = p[0]; hi[2 * w - 3] = p[1]; }
  }
}
QA_DEVICE float wave_max_abs16(const float* x) {
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) m = fmaxf(m, fabsf(x[i]));
  return wave_max_f(m);
}

// D[row] = fp16( sum_d fp32(fp16(dO*O)) ), stored as fp32 (int8:398)
template <int D>
__global__ __launch_bounds__(256) void int8_bwd_drow_kernel(const _Float16* __restrict__ dO,
                                                            const _Float16* __restrict__ O,
                                                            float* __restrict__ Drow, long rows) {
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
  if (row < rows && (threadIdx.x % LPR) == 0) Drow[row] = (float)(_Float16)acc;
}

// ------------------------------------------------------------------------- kernel A: dK, dV
template <int D>
__global__ __launch_bounds__(256, 1) void int8_bwd_dkdv_kernel(
    const int8_t* __restrict__ dOi, const _Float16* __restrict__ sdO, const int8_t* __restrict__ qi,
    const _Float16* __restrict__ sq, const int8_t* __restrict__ ki, const _Float16* __restrict__ sk,
    const int8_t* __restrict__ vi, const _Float16* __restrict__ sv, const _Float16* __restrict__ lse,
    const float* __restrict__ Drow, _Float16* __restrict__ dk, _Float16* __restrict__ dv, int BH,
    int S, float qks, float sms) {
  using C = I8BwdCfg<D>;
  constexpr int STAGE = 2 * C::T8 + 2 * C::T16 + 2 * 32 * 4 + 16;  // Qi8, dOi8, Qbf, dObf, lse, D, scalars
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nkb = (S + 127) / 128;
  int bh, kt;
  xcd_remap(blockIdx.x, nkb, BH, bh, kt);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int k0 = kt * 128 + wave * 32;
  const bool active = k0 < S;
  const long hrow = (long)bh * S;
  v4i kfr[C::NKS8], vfr[C::NKS8];
  float skw = 0.f, svw = 0.f;
  if (active) {
    const int8_t* kr = ki + (hrow + k0 + c32) * D + 16 * h;
    const int8_t* vr = vi + (hrow + k0 + c32) * D + 16 * h;
#pragma unroll
    for (int s = 0; s < C::NKS8; ++s) {
      kfr[s] = *reinterpret_cast<const v4i*>(kr + 32 * s);
      vfr[s] = *reinterpret_cast<const v4i*>(vr + 32 * s);
    }
    skw = (float)sk[(hrow + k0) / 32];
    svw = (float)sv[(hrow + k0) / 32];
  }
  v16f dka[C::NDB], dva[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) { dka[b] = v16f{}; dva[b] = v16f{}; }

  // staging: int8 Q tile and dO tile (32 x D bytes each): chunks of 16 B
  constexpr int CH8 = 32 * C::NCH8;           // chunks per int8 tile
  v4i sq8 = v4i{0, 0, 0, 0}, sd8 = v4i{0, 0, 0, 0};
  float sl = 0.f, sD = 0.f, ssc = 0.f;
  auto stage_load = [&](int t) {
    const long r0 = hrow + 32L * t;
    if (tid < CH8) {
      const int row = tid / C::NCH8, ch = tid % C::NCH8;
      sq8 = *reinterpret_cast<const v4i*>(qi + (r0 + row) * D + 16 * ch);
      sd8 = *reinterpret_cast<const v4i*>(dOi + (r0 + row) * D + 16 * ch);
    }
    if (tid < 32) sl = (float)lse[r0 + tid];
    else if (tid < 64) sD = Drow[r0 + tid - 32];
    else if (tid == 64) ssc = (float)sq[r0 / 32];
    else if (tid == 65) ssc = (float)sdO[r0 / 32];
  };
  auto stage_store = [&](int buf) {
    char* base = smem + buf * STAGE;
    char* q8 = base;
    char* d8 = base + C::T8;
    char* qb = base + 2 * C::T8;
    char* db = qb + C::T16;
    float* fl = reinterpret_cast<float*>(db + C::T16);
    if (tid < CH8) {
      const int row = tid / C::NCH8, ch = tid % C::NCH8;
      *reinterpret_cast<v4i*>(q8 + i8_off<D>(row, ch)) = sq8;
      *reinterpret_cast<v4i*>(d8 + i8_off<D>(row, ch)) = sd8;
      v4u lo, hi;
      i8x16_to_bf16(sq8, lo, hi);
      *reinterpret_cast<v4u*>(qb + t16_off<D>(row, 2 * ch)) = lo;
      *reinterpret_cast<v4u*>(qb + t16_off<D>(row, 2 * ch + 1)) = hi;
      i8x16_to_bf16(sd8, lo, hi);
      *reinterpret_cast<v4u*>(db + t16_off<D>(row, 2 * ch)) = lo;
      *reinterpret_cast<v4u*>(db + t16_off<D>(row, 2 * ch + 1)) = hi;
    }
    if (tid < 32) fl[tid] = sl;
    else if (tid < 64) fl[tid] = sD;
    else if (tid < 66) fl[tid] = ssc;
  };
  const int nqt = S / 32;
  stage_load(0);
  stage_store(0);
  __syncthreads();
  for (int t = 0; t < nqt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nqt) stage_load(t + 1);
    const char* base = smem + buf * STAGE;
    const char* q8 = base;
    const char* d8 = base + C::T8;
    const char* qb = base + 2 * C::T8;
    const char* db = qb + C::T16;
    const float* fl = reinterpret_cast<const float*>(db + C::T16);
    if (active) {
      v16i sacc = v16i{}, pacc = v16i{};
#pragma unroll
      for (int s = 0; s < C::NKS8; ++s) {
        const v4i a = *reinterpret_cast<const v4i*>(q8 + i8_off<D>(c32, 2 * s + h));
        sacc = mfma_i8(a, kfr[s], sacc);
      }
#pragma unroll
      for (int s = 0; s < C::NKS8; ++s) {
        const v4i a = *reinterpret_cast<const v4i*>(d8 + i8_off<D>(c32, 2 * s + h));
        pacc = mfma_i8(a, vfr[s], pacc);
      }
      const float sqt = fl[64], sdt = fl[65];
      float P[16], dS[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f l4 = *reinterpret_cast<const v4f*>(fl + 8 * g + 4 * h);
        const v4f d4 = *reinterpret_cast<const v4f*>(fl + 32 + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i = 4 * g + j;
          const _Float16 s16 = (_Float16)((((float)sacc[i] * sqt) * skw) * qks);
          P[i] = exp2_f32((float)(_Float16)(s16 - (_Float16)l4[j]));
          const float dp = ((float)pacc[i] * sdt) * svw;
          dS[i] = P[i] * (dp - d4[j]);
        }
      }
      const float sP = wave_max_abs16(P) / 127.0f;
      const float ssd = wave_max_abs16(dS) / 127.0f;
      const float iP = sP > 0.f ? 1.0f / sP : 0.f;
      const float iS = ssd > 0.f ? 1.0f / ssd : 0.f;
      const float cP = sP * sdt;   // dV operand scale
      const float cS = ssd * sqt;  // dK operand scale
      v8bf pb[2], sb[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        v4u pp, ss;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int i0 = 8 * s + 2 * j, i1 = i0 + 1;
          pp[j] = pk_bf16(__builtin_truncf(P[i0] * iP) * cP, __builtin_truncf(P[i1] * iP) * cP);
          ss[j] = pk_bf16(__builtin_truncf(dS[i0] * iS) * cS, __builtin_truncf(dS[i1] * iS) * cS);
        }
        pb[s] = __builtin_bit_cast(v8bf, pp);
        sb[s] = __builtin_bit_cast(v8bf, ss);
      }
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          dva[b] = mfma_bf16(t16_frag<D>(db, 16 * s, b, lane), pb[s], dva[b]);
          dka[b] = mfma_bf16(t16_frag<D>(qb, 16 * s, b, lane), sb[s], dka[b]);
        }
      }
    }
    if (t + 1 < nqt) stage_store(buf ^ 1);
    __syncthreads();
  }
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
      *reinterpret_cast<v4h*>(dk + krow * D + 32 * b + 8 * g + 4 * h) = wk;
      *reinterpret_cast<v4h*>(dv + krow * D + 32 * b + 8 * g + 4 * h) = wv;
    }
  }
}

// ----------------------------------------------------------------------------- kernel B: dQ
template <int D>
__global__ __launch_bounds__(256, 1) void int8_bwd_dq_kernel(
    const int8_t* __restrict__ dOi, const _Float16* __restrict__ sdO, const int8_t* __restrict__ qi,
    const _Float16* __restrict__ sq, const int8_t* __restrict__ ki, const _Float16* __restrict__ sk,
    const int8_t* __restrict__ vi, const _Float16* __restrict__ sv, const _Float16* __restrict__ lse,
    const float* __restrict__ Drow, _Float16* __restrict__ dq, int BH, int S, float qks, float sms) {
  using C = I8BwdCfg<D>;
  constexpr int KB = 64;
  constexpr int STAGE = 2 * KB * C::RB8 + KB * C::RB16 + 16;  // K i8, V i8, K bf16, sk/sv
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (S + 127) / 128;
  int bh, qt;
  xcd_remap(blockIdx.x, nqb, BH, bh, qt);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qt * 128 + wave * 32;
  const bool active = q0 < S;
  const long hrow = (long)bh * S;
  v4i qfr[C::NKS8], ofr[C::NKS8];
  float lq = 0.f, Dq = 0.f, sqw = 0.f, sdw = 0.f;
  if (active) {
    const long r = hrow + q0 + c32;
#pragma unroll
    for (int s = 0; s < C::NKS8; ++s) {
      qfr[s] = *reinterpret_cast<const v4i*>(qi + r * D + 16 * h + 32 * s);
      ofr[s] = *reinterpret_cast<const v4i*>(dOi + r * D + 16 * h + 32 * s);
    }
    lq = (float)lse[r];
    Dq = Drow[r];
    sqw = (float)sq[(hrow + q0) / 32];
    sdw = (float)sdO[(hrow + q0) / 32];
  }
  v16f acc[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) acc[b] = v16f{};
  constexpr int CH8 = KB * C::NCH8;          // 16-B chunks per int8 K (or V) block
  constexpr int LOADS = (CH8 + 255) / 256;
  v4i sk8[LOADS], sv8[LOADS];
  float ssc = 0.f;
  auto stage_load = [&](int kb) {
    const long r0 = hrow + (long)kb * KB;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int e = i * 256 + tid;
      if (e < CH8) {
        const int row = e / C::NCH8, ch = e % C::NCH8;
        sk8[i] = *reinterpret_cast<const v4i*>(ki + (r0 + row) * D + 16 * ch);
        sv8[i] = *reinterpret_cast<const v4i*>(vi + (r0 + row) * D + 16 * ch);
      }
    }
    if (tid < 2) ssc = (float)sk[r0 / 32 + tid];
    else if (tid < 4) ssc = (float)sv[r0 / 32 + tid - 2];
  };
  auto stage_store = [&](int buf) {
    char* k8 = smem + buf * STAGE;
    char* v8 = k8 + KB * C::RB8;
    char* kb16 = v8 + KB * C::RB8;
    float* fl = reinterpret_cast<float*>(kb16 + KB * C::RB16);
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int e = i * 256 + tid;
      if (e < CH8) {
        const int row = e / C::NCH8, ch = e % C::NCH8;
        *reinterpret_cast<v4i*>(k8 + i8_off<D>(row, ch)) = sk8[i];
        *reinterpret_cast<v4i*>(v8 + i8_off<D>(row, ch)) = sv8[i];
        v4u lo, hi;
        i8x16_to_bf16(sk8[i], lo, hi);
        *reinterpret_cast<v4u*>(kb16 + t16_off<D>(row, 2 * ch)) = lo;
        *reinterpret_cast<v4u*>(kb16 + t16_off<D>(row, 2 * ch + 1)) = hi;
      }
    }
    if (tid < 4) fl[tid] = ssc;
  };
  const int nkb = S / KB;
  stage_load(0);
  stage_store(0);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) stage_load(kb + 1);
    const char* k8 = smem + (kb & 1) * STAGE;
    const char* v8 = k8 + KB * C::RB8;
    const char* kb16 = v8 + KB * C::RB8;
    const float* fl = reinterpret_cast<const float*>(kb16 + KB * C::RB16);
    if (active) {
#pragma unroll
      for (int u = 0; u < KB / 32; ++u) {
        v16i sacc = v16i{}, pacc = v16i{};
#pragma unroll
        for (int s = 0; s < C::NKS8; ++s) {
          const v4i a = *reinterpret_cast<const v4i*>(k8 + i8_off<D>(32 * u + c32, 2 * s + h));
          sacc = mfma_i8(a, qfr[s], sacc);
        }
#pragma unroll
        for (int s = 0; s < C::NKS8; ++s) {
          const v4i a = *reinterpret_cast<const v4i*>(v8 + i8_off<D>(32 * u + c32, 2 * s + h));
          pacc = mfma_i8(a, ofr[s], pacc);
        }
        const float skt = fl[u], svt = fl[2 + u];
        const _Float16 l16 = (_Float16)lq;
        float dS[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const _Float16 s16 = (_Float16)((((float)sacc[i] * sqw) * skt) * qks);
          const float P = exp2_f32((float)(_Float16)(s16 - l16));
          const float dp = ((float)pacc[i] * sdw) * svt;
          dS[i] = P * (dp - Dq);
        }
        const float ssd = wave_max_abs16(dS) / 127.0f;
        const float iS = ssd > 0.f ? 1.0f / ssd : 0.f;
        const float cS = ssd * skt;
        v8bf sb[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v4u ss;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i0 = 8 * s + 2 * j;
            ss[j] = pk_bf16(__builtin_truncf(dS[i0] * iS) * cS, __builtin_truncf(dS[i0 + 1] * iS) * cS);
          }
          sb[s] = __builtin_bit_cast(v8bf, ss);
        }
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[b] = mfma_bf16(t16_frag<D>(kb16, 32 * u + 16 * s, b, lane), sb[s], acc[b]);
        }
      }
    }
    if (kb + 1 < nkb) stage_store((kb + 1) & 1);
    __syncthreads();
  }
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

extern "C" int qattn_int8_bwd_prep(const void* dO, const void* O, void* dO_i8, void* sdO, void* Drow,
                                   long bh, long seq, int head_dim, void* stream) {
  if (seq % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  const long rows = bh * seq;
  if (rows == 0) return 0;
  int rc = qattn_int8_quant(dO, dO_i8, sdO, nullptr, nullptr, rows, (int)seq, head_dim, stream);
  if (rc) return rc;
  const int rpb = 256 / (head_dim / 8);
  dim3 grid((unsigned)((rows + rpb - 1) / rpb)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL((int8_bwd_drow_kernel<128>), grid, block, 0, st, (const _Float16*)dO,
                       (const _Float16*)O, (float*)Drow, rows);
  else
    hipLaunchKernelGGL((int8_bwd_drow_kernel<64>), grid, block, 0, st, (const _Float16*)dO,
                       (const _Float16*)O, (float*)Drow, rows);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// which: 1 = dK/dV kernel, 2 = dQ kernel, 3 = both
static int int8_bwd_launch(int which, const void* dO_i8, const void* sdO, const void* q_i8,
                           const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                           const void* sv, const void* lse, const void* Drow, void* dq, void* dk,
                           void* dv, long bh, long seq, int head_dim, float qks, float sms,
                           void* stream) {
  if (seq % 64 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)((seq + 127) / 128);
#define QA_LAUNCH(Dv)                                                                            \
  {                                                                                              \
    using C = I8BwdCfg<Dv>;                                                                      \
    constexpr int sA = 2 * (2 * C::T8 + 2 * C::T16 + 2 * 32 * 4 + 16);                          \
    constexpr int sB = 2 * (2 * 64 * C::RB8 + 64 * C::RB16 + 16);                               \
    if (which & 1) {                                                                             \
      hipFuncSetAttribute((const void*)int8_bwd_dkdv_kernel<Dv>,                                 \
                          hipFuncAttributeMaxDynamicSharedMemorySize, sA);                       \
      hipLaunchKernelGGL((int8_bwd_dkdv_kernel<Dv>), dim3((unsigned)(nb * bh)), dim3(256), sA,    \
                         st, (const int8_t*)dO_i8, (const _Float16*)sdO, (const int8_t*)q_i8,     \
                         (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,           \
                         (const int8_t*)v_i8, (const _Float16*)sv, (const _Float16*)lse,          \
                         (const float*)Drow, (_Float16*)dk, (_Float16*)dv, (int)bh, (int)seq,     \
                         qks, sms);                                                              \
    }                                                                                            \
    if (which & 2) {                                                                             \
      hipFuncSetAttribute((const void*)int8_bwd_dq_kernel<Dv>,                                   \
                          hipFuncAttributeMaxDynamicSharedMemorySize, sB);                       \
      hipLaunchKernelGGL((int8_bwd_dq_kernel<Dv>), dim3((unsigned)(nb * bh)), dim3(256), sB, st,  \
                         (const int8_t*)dO_i8, (const _Float16*)sdO, (const int8_t*)q_i8,         \
                         (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,           \
                         (const int8_t*)v_i8, (const _Float16*)sv, (const _Float16*)lse,          \
                         (const float*)Drow, (_Float16*)dq, (int)bh, (int)seq, qks, sms);         \
    }                                                                                            \
  }
  if (head_dim == 128) QA_LAUNCH(128) else QA_LAUNCH(64)
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_attn_bwd(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* lse, const void* Drow, void* dq,
                                   void* dk, void* dv, void* ws0, void* ws1, void* ws2, long bh,
                                   long seq, int head_dim, float qks, float sms, void* stream) {
  (void)ws0; (void)ws1; (void)ws2;
  return int8_bwd_launch(3, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, lse, Drow, dq, dk, dv, bh, seq,
                         head_dim, qks, sms, stream);
}

extern "C" int qattn_int8_bwd_dkdv(const void* dO_i8, const void* sdO, const void* q_i8,
                                   const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                   const void* sv, const void* lse, const void* Drow, void* dk,
                                   void* dv, long bh, long seq, int head_dim, float qks, float sms,
                                   void* stream) {
  return int8_bwd_launch(1, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, lse, Drow, nullptr, dk, dv, bh,
                         seq, head_dim, qks, sms, stream);
}

extern "C" int qattn_int8_bwd_dq(const void* dO_i8, const void* sdO, const void* q_i8,
                                 const void* sq, const void* k_i8, const void* sk, const void* v_i8,
                                 const void* sv, const void* lse, const void* Drow, void* dq, long bh,
                                 long seq, int head_dim, float qks, float sms, void* stream) {
  return int8_bwd_launch(2, dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, lse, Drow, dq, nullptr, nullptr,
                         bh, seq, head_dim, qks, sms, stream);
}
