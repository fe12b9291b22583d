// FlashAttention-2 backward (algorithm 4) for gfx950; replaces helion_flash_atten_2_algo_4_bwd
// (attention_bf16.py:299-448) with the build-contract fixes of SURVEY F3:
//   P  = exp2(qks * q.k - lse)      (causal: strictly-lower kept, else qks*S := -128)  bf16:376-392
//   dV = P^T dO                                                                          bf16:399
//   dP = dO V^T ;  D = rowsum(dO * O) (once per row, prep kernel)                        bf16:405,416
//   dS = P * (dP - D)                (reference: S * (dP - D), F3)                       bf16:421
//   dQ = sm_scale * dS K ;  dK = sm_scale * dS^T Q   (reference: qk_scale, racy dq RMW)   bf16:427-441
//
// Deterministic by construction: kernel A owns a block of keys and accumulates dK, dV over all
// query tiles in registers; kernel B owns a block of queries and accumulates dQ over all key tiles
// (S and dP are recomputed there; no atomics, no read-modify-write of global memory).
//
// MFMA precisions: S = Q K^T in fp16 (inputs are fp16, products exact, fp32 accumulate);
// dP, dV, dK, dQ in bf16 (dO, dS rounded to bf16; Q/K rounded to bf16 for the dK/dQ products;
// V is bf16 already), fp32 accumulate.  Causal tiles that are entirely masked contribute
// exp2(-128 - lse) < 2^-120 per element and are skipped.
#include "common.h"

namespace qattn {

// ------------------------------------------------------------------------------------------ prep
// D[row] = sum_d dO*O (fp32);  dO_bf16 = bf16(dO).   16 lanes per row, 8 floats per lane (D=128).
template <int D>
__global__ __launch_bounds__(256) void bf16_bwd_prep_kernel(const float* __restrict__ dO,
                                                            const float* __restrict__ O,
                                                            __bf16* __restrict__ dO_bf,
                                                            float* __restrict__ Drow, long rows) {
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
  if (row < rows && (threadIdx.x % LPR) == 0) Drow[row] = acc;
}

template <int D>
struct BwdCfg {
  static constexpr int ROWB = 2 * D;     // bytes per 16-bit row
  static constexpr int NCH = ROWB / 16;
  static constexpr int NKS = D / 16;     // 32x32x16 k-steps over D
  static constexpr int NDB = D / 32;
};
// One LDS image serves row reads (ds_read_b128) and transposed reads (ds_read_b64_tr_b16) of the
// same tile; the 16-B chunk swizzle is conflict-free for both (bank model of MI355X_MICROARCH §LDS):
//   D=128 (256-B rows): ch ^ (((row&3)<<2) | ((row>>2)&3))      (cdna_hip_programming.md T10 (b))
//   D=64  (128-B rows): ch ^ (((row&3)<<1) ^ ((row>>2)&3))
template <int D>
QA_DEVICE int img_off(int row, int ch) {
  using C = BwdCfg<D>;
  const int sw = (D == 128) ? (((row & 3) << 2) | ((row >> 2) & 3))
                            : ((((row & 3) << 1) ^ ((row >> 2) & 3)) & 7);
  return row * C::ROWB + 16 * (ch ^ sw);
}
// A operand (X^T, 32 d x 16 rows) of a 32x32x16 product from a row-major [row][d] tile.
template <int D>
QA_DEVICE v8s tr_frag(const char* base, int row_base, int b, int lane) {
  const int h = lane >> 5, gg = (lane >> 4) & 1, i16 = lane & 15;
  const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
  const int row = row_base + 4 * h + (i16 >> 2);
  const int ch = d / 8, within = (d % 8) * 2;
  return ds_read_tr16_x2(base + img_off<D>(row, ch) + within, base + img_off<D>(row + 8, ch) + within);
}

// ------------------------------------------------------------------------- kernel A: dK, dV
// Workgroup = 4 waves x 32 keys (128 keys of one head); loops over 32-row query tiles staged in
// LDS: Q fp16 (row image for S), Q bf16 (tr image for dK), dO bf16 (row image for dP, tr image for
// dV), lse and D.  Orientation: query rows in registers, key on the lane.
template <int D>
__global__ __launch_bounds__(256, 1) void bf16_bwd_dkdv_kernel(
    const _Float16* __restrict__ q, const _Float16* __restrict__ k, const __bf16* __restrict__ v,
    const __bf16* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ Drow,
    float* __restrict__ dk, float* __restrict__ dv, int BH, int Sq, int Sk, int causal, float qks,
    float sms) {
  using C = BwdCfg<D>;
  constexpr int TQ = 32 * C::ROWB;           // one 32-row 16-bit tile
  constexpr int STAGE = 3 * TQ + 2 * 32 * 4; // Qh, Qb, dO, lse, D
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nkb = (Sk + 127) / 128;
  int bh, kt;
  xcd_remap(blockIdx.x, nkb, BH, bh, kt);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int k0 = kt * 128 + wave * 32;
  const bool active = k0 < Sk;
  const int key = k0 + c32;

  // K (fp16) and V (bf16) fragments as B operands: lane holds row `key`, d = 16s + 8h .. +8
  v8h kf[C::NKS];
  v8bf vf[C::NKS];
  if (active) {
    const _Float16* kr = k + ((long)bh * Sk + key) * D + 8 * h;
    const __bf16* vr = v + ((long)bh * Sk + key) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
      kf[s] = *reinterpret_cast<const v8h*>(kr + 16 * s);
      vf[s] = *reinterpret_cast<const v8bf*>(vr + 16 * s);
    }
  }
  v16f dka[C::NDB], dva[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) { dka[b] = v16f{}; dva[b] = v16f{}; }

  const long qrow0 = (long)bh * Sq;
  const int nqt = Sq / 32;
  int qt0 = 0;
  if (causal) qt0 = min(nqt, (kt * 128) / 32);  // tiles with q_max <= k_min are fully masked
  // staging: 3 tiles x 32 rows x NCH chunks of 16 B -> per thread (3*32*NCH)/256 chunks
  constexpr int CH_PER_TILE = 32 * C::NCH;
  constexpr int LOADS = (CH_PER_TILE + 255) / 256;
  v4i sq_[LOADS], sd_[LOADS];
  float slse = 0.f, sD = 0.f;
  auto stage_load = [&](int t) {
    const long r0 = qrow0 + 32L * t;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int e = i * 256 + tid;
      if (e < CH_PER_TILE) {
        const int row = e / C::NCH, ch = e % C::NCH;
        sq_[i] = *reinterpret_cast<const v4i*>(reinterpret_cast<const char*>(q + (r0 + row) * D) + 16 * ch);
        sd_[i] = *reinterpret_cast<const v4i*>(reinterpret_cast<const char*>(dO + (r0 + row) * D) + 16 * ch);
      }
    }
    if (tid < 32) slse = lse[r0 + tid];
    else if (tid < 64) sD = Drow[r0 + tid - 32];
  };
  auto stage_store = [&](int buf) {
    char* base = smem + buf * STAGE;
    char* qh = base;
    char* qb = base + TQ;
    char* dd = base + 2 * TQ;
    float* ls = reinterpret_cast<float*>(base + 3 * TQ);
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int e = i * 256 + tid;
      if (e < CH_PER_TILE) {
        const int row = e / C::NCH, ch = e % C::NCH;
        *reinterpret_cast<v4i*>(qh + img_off<D>(row, ch)) = sq_[i];
        *reinterpret_cast<v4i*>(dd + img_off<D>(row, ch)) = sd_[i];
        // fp16 -> bf16 copy of Q for the dK product
        const v8h x = __builtin_bit_cast(v8h, sq_[i]);
        v4u pk;
#pragma unroll
        for (int j = 0; j < 4; ++j) pk[j] = pk_bf16((float)x[2 * j], (float)x[2 * j + 1]);
        *reinterpret_cast<v4u*>(qb + img_off<D>(row, ch)) = pk;
      }
    }
    if (tid < 32) ls[tid] = slse;
    else if (tid < 64) ls[tid] = sD;
  };

  if (qt0 < nqt) {
    stage_load(qt0);
    stage_store(0);
  }
  __syncthreads();
  for (int t = qt0; t < nqt; ++t) {
    const int buf = (t - qt0) & 1;
    if (t + 1 < nqt) stage_load(t + 1);
    const char* base = smem + buf * STAGE;
    const char* qh = base;
    const char* qb = base + TQ;
    const char* dd = base + 2 * TQ;
    const float* ls = reinterpret_cast<const float*>(base + 3 * TQ);
    const int qtile0 = 32 * t;
    const bool skip = causal && (qtile0 + 31 <= k0);  // fully masked for this wave's keys
    if (active && !skip) {
      // S[q][key] = Q K^T (fp16) and dP[q][key] = dO V^T (bf16); q rows in registers
      v16f sacc = v16f{}, pacc = v16f{};
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const v8h a = *reinterpret_cast<const v8h*>(qh + img_off<D>(c32, 2 * s + h));
        sacc = mfma_f16(a, kf[s], sacc);
      }
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const v8bf a = *reinterpret_cast<const v8bf*>(dd + img_off<D>(c32, 2 * s + h));
        pacc = mfma_bf16(a, vf[s], pacc);
      }
      // row constants for rows (r&3) + 8(r>>2) + 4h: 4 contiguous floats per group g
      float lr[16], dr[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f l4 = *reinterpret_cast<const v4f*>(ls + 8 * g + 4 * h);
        const v4f d4 = *reinterpret_cast<const v4f*>(ls + 32 + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) { lr[4 * g + j] = l4[j]; dr[4 * g + j] = d4[j]; }
      }
      const bool need_mask = causal && (qtile0 <= k0 + 31);
      float p[16], ds[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float sc = sacc[i] * qks;
        if (need_mask) {
          const int qi = qtile0 + (i & 3) + 8 * (i >> 2) + 4 * h;
          if (qi - key <= 0) sc = -128.0f;
        }
        p[i] = exp2_f32(sc - lr[i]);
        ds[i] = p[i] * (pacc[i] - dr[i]);
      }
      v8bf pb[2], db[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        v4u pp, dq;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pp[j] = pk_bf16(p[8 * s + 2 * j], p[8 * s + 2 * j + 1]);
          dq[j] = pk_bf16(ds[8 * s + 2 * j], ds[8 * s + 2 * j + 1]);
        }
        pb[s] = __builtin_bit_cast(v8bf, pp);
        db[s] = __builtin_bit_cast(v8bf, dq);
      }
      // dV^T[d][key] += dO^T P ;  dK^T[d][key] += Q^T dS
#pragma unroll
      for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const v8bf ao = __builtin_bit_cast(v8bf, tr_frag<D>(dd, 16 * s, b, lane));
          dva[b] = mfma_bf16(ao, pb[s], dva[b]);
          const v8bf aq = __builtin_bit_cast(v8bf, tr_frag<D>(qb, 16 * s, b, lane));
          dka[b] = mfma_bf16(aq, db[s], dka[b]);
        }
      }
    }
    if (t + 1 < nqt) stage_store(buf ^ 1);
    __syncthreads();
  }
  if (!active) return;
  // write dK = sms * dK^T, dV (fp32, row-major [key][d]); lane = key, regs = d
  const long krow = (long)bh * Sk + key;
  float* dkr = dk + krow * D;
  float* dvr = dv + krow * D;
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4f wk, wv;
#pragma unroll
      for (int j = 0; j < 4; ++j) { wk[j] = dka[b][4 * g + j] * sms; wv[j] = dva[b][4 * g + j]; }
      *reinterpret_cast<v4f*>(dkr + 32 * b + 8 * g + 4 * h) = wk;
      *reinterpret_cast<v4f*>(dvr + 32 * b + 8 * g + 4 * h) = wv;
    }
  }
}

// ----------------------------------------------------------------------------- kernel B: dQ
// Workgroup = 4 waves x 32 queries; loops over 64-key blocks staged in LDS: K fp16 (row image for
// S), K bf16 (tr image for dQ), V bf16 (row image for dP).  Orientation: keys in registers, query
// on the lane (lse, D are per-lane scalars).
template <int D>
__global__ __launch_bounds__(256, 1) void bf16_bwd_dq_kernel(
    const _Float16* __restrict__ q, const _Float16* __restrict__ k, const __bf16* __restrict__ v,
    const __bf16* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ Drow,
    float* __restrict__ dq, int BH, int Sq, int Sk, int causal, float qks, float sms) {
  using C = BwdCfg<D>;
  constexpr int KB = 64;
  constexpr int TK = KB * C::ROWB;
  constexpr int STAGE = 3 * TK;  // Kh, Kb, V
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nqb = (Sq + 127) / 128;
  int bh, qt;
  xcd_remap(blockIdx.x, nqb, BH, bh, qt);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qt * 128 + wave * 32;
  const bool active = q0 < Sq;
  const int qi = q0 + c32;

  v8h qf[C::NKS];
  v8bf of[C::NKS];
  float lq = 0.f, dq_ = 0.f;
  if (active) {
    const long r = (long)bh * Sq + qi;
    const _Float16* qr = q + r * D + 8 * h;
    const __bf16* orr = dO + r * D + 8 * h;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) {
      qf[s] = *reinterpret_cast<const v8h*>(qr + 16 * s);
      of[s] = *reinterpret_cast<const v8bf*>(orr + 16 * s);
    }
    lq = lse[r];
    dq_ = Drow[r];
  }
  v16f acc[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) acc[b] = v16f{};

  int nkb = (Sk + KB - 1) / KB;
  if (causal) nkb = min(nkb, (qt * 128 + 127 + KB - 1) / KB);  // blocks with k_min >= q_max skipped
  constexpr int CH = KB * C::NCH;
  constexpr int LOADS = CH / 256;
  v4i sk_[LOADS], sv_[LOADS];
  const char* kbase = reinterpret_cast<const char*>(k + (long)bh * Sk * D);
  const char* vbase = reinterpret_cast<const char*>(v + (long)bh * Sk * D);
  auto stage_load = [&](int kb) {
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int e = i * 256 + tid, row = e / C::NCH, ch = e % C::NCH;
      const long off = (long)(kb * KB + row) * C::ROWB + 16 * ch;
      sk_[i] = *reinterpret_cast<const v4i*>(kbase + off);
      sv_[i] = *reinterpret_cast<const v4i*>(vbase + off);
    }
  };
  auto stage_store = [&](int buf) {
    char* kh = smem + buf * STAGE;
    char* kb_ = kh + TK;
    char* vl = kh + 2 * TK;
#pragma unroll
    for (int i = 0; i < LOADS; ++i) {
      const int e = i * 256 + tid, row = e / C::NCH, ch = e % C::NCH;
      *reinterpret_cast<v4i*>(kh + img_off<D>(row, ch)) = sk_[i];
      *reinterpret_cast<v4i*>(vl + img_off<D>(row, ch)) = sv_[i];
      const v8h x = __builtin_bit_cast(v8h, sk_[i]);
      v4u pk;
#pragma unroll
      for (int j = 0; j < 4; ++j) pk[j] = pk_bf16((float)x[2 * j], (float)x[2 * j + 1]);
      *reinterpret_cast<v4u*>(kb_ + img_off<D>(row, ch)) = pk;
    }
  };
  if (nkb > 0) {
    stage_load(0);
    stage_store(0);
  }
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 1 < nkb) stage_load(kb + 1);
    const char* kh = smem + (kb & 1) * STAGE;
    const char* kbf = kh + TK;
    const char* vl = kh + 2 * TK;
    if (active) {
#pragma unroll
      for (int u = 0; u < KB / 32; ++u) {
        const int key_t0 = kb * KB + 32 * u;
        if (causal && key_t0 >= q0 + 31) continue;  // fully masked for this wave (uniform)
        v16f sacc = v16f{}, pacc = v16f{};
#pragma unroll
        for (int s = 0; s < C::NKS; ++s) {
          const v8h a = *reinterpret_cast<const v8h*>(kh + img_off<D>(32 * u + c32, 2 * s + h));
          sacc = mfma_f16(a, qf[s], sacc);
        }
#pragma unroll
        for (int s = 0; s < C::NKS; ++s) {
          const v8bf a = *reinterpret_cast<const v8bf*>(vl + img_off<D>(32 * u + c32, 2 * s + h));
          pacc = mfma_bf16(a, of[s], pacc);
        }
        const bool need_mask = causal && (key_t0 + 31 >= q0);
        float ds[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float sc = sacc[i] * qks;
          if (need_mask) {
            const int kk = key_t0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (qi - kk <= 0) sc = -128.0f;
          }
          const float p = exp2_f32(sc - lq);
          ds[i] = p * (pacc[i] - dq_);
        }
        v8bf db[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          v4u pk;
#pragma unroll
          for (int j = 0; j < 4; ++j) pk[j] = pk_bf16(ds[8 * s + 2 * j], ds[8 * s + 2 * j + 1]);
          db[s] = __builtin_bit_cast(v8bf, pk);
        }
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const v8bf a = __builtin_bit_cast(v8bf, tr_frag<D>(kbf, 32 * u + 16 * s, b, lane));
            acc[b] = mfma_bf16(a, db[s], acc[b]);
          }
        }
      }
    }
    if (kb + 1 < nkb) stage_store((kb + 1) & 1);
    __syncthreads();
  }
  if (!active) return;
  float* dqr = dq + ((long)bh * Sq + qi) * D;
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      v4f w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = acc[b][4 * g + j] * sms;
      *reinterpret_cast<v4f*>(dqr + 32 * b + 8 * g + 4 * h) = w;
    }
  }
}

template <typename K>
static void set_lds(K kernel, int bytes) {
  hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_bf16_bwd_prep(const void* dO, const void* O, void* dO_bf, void* Drow, long bh,
                                   long seq, int head_dim, void* stream) {
  if (head_dim != 64 && head_dim != 128) return 1;
  const long rows = bh * seq;
  if (rows == 0) return 0;
  const int rpb = 256 / (head_dim / 8);
  dim3 grid((unsigned)((rows + rpb - 1) / rpb)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL((bf16_bwd_prep_kernel<128>), grid, block, 0, st, (const float*)dO,
                       (const float*)O, (__bf16*)dO_bf, (float*)Drow, rows);
  else
    hipLaunchKernelGGL((bf16_bwd_prep_kernel<64>), grid, block, 0, st, (const float*)dO,
                       (const float*)O, (__bf16*)dO_bf, (float*)Drow, rows);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_bf16_bwd(const void* q, const void* k, const void* v, const void* dO_bf,
                              const void* lse, const void* Drow, void* dq, void* dk, void* dv,
                              long bh, long sq, long sk, int head_dim, int causal, float qks,
                              float sms, void* stream) {
  if (sq % 32 != 0 || sk % 64 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0 || sq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int nkb = (int)((sk + 127) / 128), nqb = (int)((sq + 127) / 128);
#define QA_LAUNCH(Dv)                                                                              \
  {                                                                                                \
    constexpr int sA = 2 * (3 * 32 * 2 * Dv + 256);                                                \
    constexpr int sB = 2 * 3 * 64 * 2 * Dv;                                                        \
    set_lds(bf16_bwd_dkdv_kernel<Dv>, sA);                                                         \
    set_lds(bf16_bwd_dq_kernel<Dv>, sB);                                                           \
    hipLaunchKernelGGL((bf16_bwd_dkdv_kernel<Dv>), dim3((unsigned)(nkb * bh)), dim3(256), sA, st,   \
                       (const _Float16*)q, (const _Float16*)k, (const __bf16*)v,                     \
                       (const __bf16*)dO_bf, (const float*)lse, (const float*)Drow, (float*)dk,      \
                       (float*)dv, (int)bh, (int)sq, (int)sk, causal, qks, sms);                    \
    hipLaunchKernelGGL((bf16_bwd_dq_kernel<Dv>), dim3((unsigned)(nqb * bh)), dim3(256), sB, st,     \
                       (const _Float16*)q, (const _Float16*)k, (const __bf16*)v,                     \
                       (const __bf16*)dO_bf, (const float*)lse, (const float*)Drow, (float*)dq,      \
                       (int)bh, (int)sq, (int)sk, causal, qks, sms);                                 \
  }
  if (head_dim == 128) QA_LAUNCH(128) else QA_LAUNCH(64)
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
