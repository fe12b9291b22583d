// SageAttention-3 int8 attention forward for gfx950 (replaces the attention part of
// helion_atten_int8_hl_dot_fwd, attention_int8.py:170-257), per (batch, head).
//
// Work decomposition
//   * one workgroup = 4 waves = 128 query rows of one (b,h); wave w owns rows 32w..32w+31, which is
//     exactly one 32-token q-quant block (one sq scale per wave);
//   * keys stream in 64-key blocks (two 32-key Bkv tiles) through a 2-stage LDS ring
//     (register staging: issue global loads for block j+1, compute block j, write LDS, 1 barrier);
//   * workgroups of one head are kept on one XCD (K/V of a head stay in that XCD's L2).
//
// Per 32-key tile and wave (the "swapped" orientation: keys in registers, queries on lanes):
//   S^T[key][q] = K_i8 . Q_i8^T          4 x v_mfma_i32_32x32x32_i8  (D=128)
//   per-q online softmax in registers (no LDS):
//     S   = fp16(acc * sq*sk*qks)                         (int8:200-203)
//     m'  = max(m, rowmax S);  P = exp2(fp16(S - m'))      (int8:205-213)
//     r   = exp2(fp16(m - m')); l = l*r + sum P; O *= r    (int8:217-225)
//     sp  = exp2(fp16(rowmax S - m')) / 127; P_i8 = trunc(P / sp)   (int8:232-237)
//   O^T[d][q] += Vdq^T . (P_i8*sp)^T       8 x v_mfma_f32_32x32x16_f16 (D=128)
// where Vdq = fp16(v_i8 * sv) is written by the quantiser.  Sum_t sp*sv*(P_i8 . v_i8) of the
// reference (int8:249-250) is computed exactly up to the fp16 rounding of the two dequantised
// operands (relative 2^-12 each); the fp32 accumulation then runs inside the MFMA, which removes
// the per-tile i32->f32 dequantisation of a D-wide accumulator (8 VALU ops per score element).
#include "common.h"

namespace qattn {

template <int D>
struct Int8FwdCfg {
  static constexpr int KB = 64;                 // keys per LDS stage
  static constexpr int K_BYTES = KB * D;        // int8 K block
  static constexpr int V_BYTES = KB * D * 2;    // fp16 Vdq block
  static constexpr int STAGE = K_BYTES + V_BYTES;
  static constexpr int NKS = D / 32;            // i8 k-steps for QK^T
  static constexpr int NDB = D / 32;            // 32-wide d blocks of O^T
  static constexpr int K_CH = D / 16;           // 16-B chunks per K row
  static constexpr int V_CH = D * 2 / 16;       // 16-B chunks per V row
  static constexpr int K_SW_SHIFT = (D == 128) ? 1 : 2;
  static constexpr int V_SW_SHIFT = (D == 128) ? 2 : 1;
  static constexpr int K_LOADS = K_BYTES / (256 * 16);   // dwordx4 per thread
  static constexpr int V_LOADS = V_BYTES / (256 * 16);
};

template <int D>
QA_DEVICE int k_lds_off(int row, int ch) {
  using C = Int8FwdCfg<D>;
  return row * D + 16 * (ch ^ ((row >> C::K_SW_SHIFT) & (C::K_CH - 1)));
}
template <int D>
QA_DEVICE int v_lds_off(int row, int ch) {
  using C = Int8FwdCfg<D>;
  return row * (2 * D) + 16 * (ch ^ ((row & 3) << C::V_SW_SHIFT));
}

template <int D, bool DBG = false>
__global__ __launch_bounds__(256, 2) void int8_attn_fwd_kernel(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const _Float16* __restrict__ vdq, _Float16* __restrict__ out,
    _Float16* __restrict__ lse, int BH, int S, float qks, float* __restrict__ dbg = nullptr) {
  using C = Int8FwdCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nq = (S + 127) / 128;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int q0 = qt * 128 + wave * 32;          // first query row of this wave
  const bool active = q0 < S;                   // wave-uniform
  const long head_row0 = (long)bh * S;

  // ---- Q fragment (B operand of S^T = K Q^T): lane holds Q[q0+c32][32s + 16h .. +16]
  v4i qf[C::NKS];
  float sqw = 0.f;
  if (active) {
    const int8_t* qrow = q_i8 + (head_row0 + q0 + c32) * D + 16 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v4i*>(qrow + 32 * s);
    sqw = (float)sq[(head_row0 + q0) / 32];
  }

  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  _Float16 m = (_Float16)(-INFINITY);
  float l = 1.0f;

  const int nkb = (S + C::KB - 1) / C::KB;
  const int8_t* kbase = k_i8 + head_row0 * D;
  const _Float16* vbase = vdq + head_row0 * D;
  const _Float16* skbase = sk + head_row0 / 32;

  // ---- register staging of one 64-key block
  v4i kst[C::K_LOADS], vst[C::V_LOADS];
  auto stage_load = [&](int kb) {
    const int key0 = kb * C::KB;
#pragma unroll
    for (int i = 0; i < C::K_LOADS; ++i) {
      const int e = (i * 256 + tid);            // 16-B chunk index within the block
      const int row = e / C::K_CH;
      if (key0 + row < S)
        kst[i] = *reinterpret_cast<const v4i*>(kbase + (long)(key0 + row) * D + 16 * (e % C::K_CH));
      else
        kst[i] = v4i{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < C::V_LOADS; ++i) {
      const int e = (i * 256 + tid);
      const int row = e / C::V_CH;
      if (key0 + row < S)
        vst[i] = *reinterpret_cast<const v4i*>(vbase + (long)(key0 + row) * D + 8 * (e % C::V_CH));
      else
        vst[i] = v4i{0, 0, 0, 0};
    }
  };
  auto stage_store = [&](int buf) {
    char* kl = smem + buf * C::STAGE;
    char* vl = kl + C::K_BYTES;
#pragma unroll
    for (int i = 0; i < C::K_LOADS; ++i) {
      const int e = (i * 256 + tid);
      *reinterpret_cast<v4i*>(kl + k_lds_off<D>(e / C::K_CH, e % C::K_CH)) = kst[i];
    }
#pragma unroll
    for (int i = 0; i < C::V_LOADS; ++i) {
      const int e = (i * 256 + tid);
      *reinterpret_cast<v4i*>(vl + v_lds_off<D>(e / C::V_CH, e % C::V_CH)) = vst[i];
    }
  };

  stage_load(0);
  stage_store(0);
  __syncthreads();

  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) stage_load(kb + 1);
    const char* kl = smem + (kb & 1) * C::STAGE;
    const char* vl = kl + C::K_BYTES;
    const int ntile = min(2, (S - kb * C::KB) / 32);
    if (active) {
      for (int u = 0; u < ntile; ++u) {
        // ---------------- S^T = K Q^T (int8 MFMA)
        v16i acc = v16i{};
#pragma unroll
        for (int s = 0; s < C::NKS; ++s) {
          const v4i kf = *reinterpret_cast<const v4i*>(kl + k_lds_off<D>(32 * u + c32, 2 * s + h));
          acc = mfma_i8(kf, qf[s], acc);
        }
        // ---------------- online softmax + per-row P quantisation (lane = query row)
        const float skt = (float)skbase[kb * 2 + u];
        const float cs = (sqw * skt) * qks;
        _Float16 s16[16];
        _Float16 rml = (_Float16)(-INFINITY);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          s16[i] = (_Float16)((float)acc[i] * cs);
          rml = (s16[i] > rml) ? s16[i] : rml;
        }
        const _Float16 rmo = (_Float16)xor32_f((float)rml);
        const _Float16 rm = rml > rmo ? rml : rmo;
        const _Float16 nm = m > rm ? m : rm;
        const float r = exp2_f32((float)(_Float16)(m - nm));
        m = nm;
        float lt = 0.f;
        float p32[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          p32[i] = exp2_f32((float)(_Float16)(s16[i] - nm));
          lt += p32[i];
        }
        lt += xor32_f(lt);
        l = l * r + lt;
        const float e = exp2_f32((float)(_Float16)(rm - nm));
        const float sp = e / 127.0f;
        const float inv = 127.0f / e;
        v8h pb[2];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float t = __builtin_truncf(p32[i] * inv);
          pb[i >> 3][i & 7] = (_Float16)(t * sp);
        }
        // ---------------- rescale O (exact no-op when r == 1 for every row of the wave)
        if (__ballot(r != 1.0f)) {
#pragma unroll
          for (int b = 0; b < C::NDB; ++b) o[b] *= r;
        }
        // ---------------- O^T += Vdq^T P^T (fp16 MFMA, fp32 accumulate)
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const int gg = (lane >> 4) & 1, i16 = lane & 15;
            const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
            const int key_a = 32 * u + 16 * s + 4 * h + (i16 >> 2);
            const int ch = d / 8, within = (d % 8) * 2;
            const v8h a = __builtin_bit_cast(
                v8h, ds_read_tr16_x2(vl + v_lds_off<D>(key_a, ch) + within,
                                     vl + v_lds_off<D>(key_a + 8, ch) + within));
            o[b] = mfma_f16(a, pb[s], o[b]);
            if constexpr (DBG) {
              if (blockIdx.x == 0 && wave == 0 && kb == 0 && u == 0 && b == 0 && s == 0) {
                for (int i = 0; i < 16; ++i) dbg[lane * 16 + i] = (float)acc[i];
                for (int i = 0; i < 16; ++i) dbg[1024 + lane * 16 + i] = (float)pb[i >> 3][i & 7];
                for (int j = 0; j < 8; ++j) dbg[2048 + lane * 8 + j] = (float)a[j];
              }
            }
          }
        }
      }
    }
    if (kb + 1 < nkb) stage_store((kb + 1) & 1);
    __syncthreads();
  }

  if (!active) return;
  // ---------------- epilogue: lse = fp16(m + fp16(log2 l)); O = fp16(O / l)   (int8:252-257)
  const long qrow = head_row0 + q0 + c32;
  if (h == 0) lse[qrow] = (_Float16)((float)m + (float)(_Float16)log2_f32(l));
  const float il = 1.0f / l;
  _Float16* orow = out + qrow * D;
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4h w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (_Float16)(o[b][4 * g + j] / l);
      *reinterpret_cast<v4h*>(orow + 32 * b + 8 * g + 4 * h) = w;
    }
  }
  (void)il;
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_probe_int8_attn_dbg(const void* q_i8, const void* sq, const void* k_i8,
                                         const void* sk, const void* vdq, void* out, void* lse,
                                         long bh, long seq, float qks, void* dbg, void* stream) {
  const int nq = (int)((seq + 127) / 128);
  hipLaunchKernelGGL((int8_attn_fwd_kernel<64, true>), dim3((unsigned)(nq * bh)), dim3(256),
                     2 * Int8FwdCfg<64>::STAGE, (hipStream_t)stream, (const int8_t*)q_i8,
                     (const _Float16*)sq, (const int8_t*)k_i8, (const _Float16*)sk,
                     (const _Float16*)vdq, (_Float16*)out, (_Float16*)lse, (int)bh, (int)seq, qks,
                     (float*)dbg);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_attn_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                                   const void* vdq, void* out, void* lse, long bh, long seq,
                                   int head_dim, float qks, void* stream) {
  if (seq % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0 || seq == 0) return 0;
  const int nq = (int)((seq + 127) / 128);
  dim3 grid((unsigned)(nq * bh)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128) {
    hipLaunchKernelGGL((int8_attn_fwd_kernel<128>), grid, block, 2 * Int8FwdCfg<128>::STAGE, st,
                       (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8,
                       (const _Float16*)sk, (const _Float16*)vdq, (_Float16*)out, (_Float16*)lse,
                       (int)bh, (int)seq, qks);
  } else {
    hipLaunchKernelGGL((int8_attn_fwd_kernel<64>), grid, block, 2 * Int8FwdCfg<64>::STAGE, st,
                       (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8,
                       (const _Float16*)sk, (const _Float16*)vdq, (_Float16*)out, (_Float16*)lse,
                       (int)bh, (int)seq, qks);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
