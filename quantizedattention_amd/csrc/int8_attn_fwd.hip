// SageAttention-3 int8 attention forward for gfx950 (replaces the attention part of
// helion_atten_int8_hl_dot_fwd, attention_int8.py:170-257), per (batch, head).
//
// Work decomposition
//   * one workgroup = 8 waves = 256 query rows of one (b,h); wave w owns rows 32w..32w+31 = one
//     32-token q-quant block (one sq scale per wave).  Two waves per SIMD: one wave's softmax VALU
//     overlaps the other's MFMAs.
//   * keys stream in 64-key blocks (two 32-key Bkv tiles) through a 2-stage LDS ring filled by
//     LDS-DMA (global_load_lds_dwordx4: no staging registers; the bank swizzle is applied to the
//     per-lane source address, the LDS image is written lane-linearly).  One barrier per block.
//   * every sk scale of the head sits in LDS (loaded once); workgroups of one head share an XCD.
//
// Per 32-key tile and wave (swapped orientation: keys in registers, query on the lane pair l, l^32):
//   S^T[key][q] = K_i8 . Q_i8^T          D/32 x v_mfma_i32_32x32x32_i8
//   per-q online softmax in packed fp16 (v_pk_*_f16, v_exp_f16), reference rounding points:
//     S    = fp16(acc * sq*sk*qks)                       (int8:200-203)
//     rm   = rowmax S;  m' = max(m, rm)                   (int8:205-209)
//     e    = exp2(fp16(S - rm))  so that P = e*exp2(rm-m') and P/sp = 127*e   (int8:211,232-236)
//     r    = exp2(fp16(m - m')); l = l*r + exp2(rm-m') * sum e;  O *= r      (int8:215-225)
//     P_i8 = trunc(127*e);  operand = fp16(P_i8 * sp), sp = exp2(rm - m')/127  (int8:232-237)
//   O^T[d][q] += Vdq^T . operand^T        2*D/32 x v_mfma_f32_32x32x16_f16
// Vdq = fp16(v_i8 * sv) is written by the quantiser, so the fp32 accumulation of
// sum_t sp*sv*(P_i8 . v_i8) (int8:249-250) runs inside the MFMA: exact up to the fp16 rounding of
// the two dequantised operands (2^-12 relative each), and the D-wide per-tile i32->f32
// dequantisation (8 VALU ops per score element) disappears.
#include "common.h"

namespace qattn {

template <int D>
struct Int8FwdCfg {
  static constexpr int WAVES = 4;
  static constexpr int QROWS = 32 * WAVES;      // query rows per workgroup
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
  static constexpr int K_INST = K_BYTES / 1024; // 1-KiB LDS-DMA wave instructions per block
  static constexpr int V_INST = V_BYTES / 1024;
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

// Issue the LDS-DMA of one 64-key block (rows >= S are clamped to a valid row; never consumed).
template <int D>
QA_DEVICE void stage_block(const int8_t* kbase, const _Float16* vbase, char* kl, int key0, int S,
                           int wave, int lane) {
  using C = Int8FwdCfg<D>;
  char* vl = kl + C::K_BYTES;
  for (int inst = wave; inst < C::K_INST; inst += C::WAVES) {
    constexpr int RPI = 64 / C::K_CH;
    const int row = inst * RPI + lane / C::K_CH, p = lane % C::K_CH;
    const int grow = min(key0 + row, S - 1);
    glds16(kbase + (long)grow * D + 16 * (p ^ k_sw<D>(row)), kl + inst * 1024);
  }
  for (int inst = wave; inst < C::V_INST; inst += C::WAVES) {
    constexpr int RPI = 64 / C::V_CH;
    const int row = inst * RPI + lane / C::V_CH, p = lane % C::V_CH;
    const int grow = min(key0 + row, S - 1);
    glds16(reinterpret_cast<const char*>(vbase + (long)grow * D) + 16 * (p ^ v_sw<D>(row)),
           vl + inst * 1024);
  }
}

// AB (diagnostic timing builds only, never dispatched by the API): 1 = no softmax VALU,
// 2 = no PV MFMA, 3 = no QK^T MFMA, 4 = no K/V streaming (LDS block 0 reused, no barriers),
// 5 = 4 + no softmax.  Outputs of AB != 0 are meaningless.
template <int D, int AB = 0>
__global__ __launch_bounds__(256, 3) void int8_attn_fwd_kernel(
    const int8_t* __restrict__ q_i8, const _Float16* __restrict__ sq, const int8_t* __restrict__ k_i8,
    const _Float16* __restrict__ sk, const _Float16* __restrict__ vdq, _Float16* __restrict__ out,
    _Float16* __restrict__ lse, int BH, int S, float qks) {
  using C = Int8FwdCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  _Float16* sk_lds = reinterpret_cast<_Float16*>(smem + 2 * C::STAGE);

  const int nq = (S + C::QROWS - 1) / C::QROWS;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int q0 = qt * C::QROWS + wave * 32;
  const bool active = q0 < S;
  const long head_row0 = (long)bh * S;
  const int8_t* kbase = k_i8 + head_row0 * D;
  const _Float16* vbase = vdq + head_row0 * D;
  const int nkb = (S + C::KB - 1) / C::KB;

  stage_block<D>(kbase, vbase, smem, 0, S, wave, lane);
  for (int i = tid; i < S / 32; i += 64 * C::WAVES) sk_lds[i] = sk[head_row0 / 32 + i];

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

  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  _Float16 m = (_Float16)(-INFINITY);
  float l = 0.f;  // the reference starts at 1.0 and wipes it with r = 0 on the first tile
  const v2h k127 = {(_Float16)127.0f, (_Float16)127.0f};
  const v2h one2 = {(_Float16)1.0f, (_Float16)1.0f};

  // lane-constant LDS byte offsets (the swizzles depend only on row bits fixed per lane):
  //   K A-operand chunk (2s+h) of row c32 (+32*D for the second tile)
  //   V^T A-operand, d-block b: key rows 4h + (i16>>2) (+16 per k-step, +8 for the 2nd read,
  //   +32 per tile), columns 32b + 16gg + 4(i16&3)
  int koff[C::NKS], voff[C::NDB];
#pragma unroll
  for (int s = 0; s < C::NKS; ++s) koff[s] = c32 * D + 16 * ((2 * s + h) ^ k_sw<D>(c32));
  {
    const int gg = (lane >> 4) & 1, i16 = lane & 15;
    const int key_a = 4 * h + (i16 >> 2);
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const int d = 32 * b + 16 * gg + 4 * (i16 & 3);
      voff[b] = key_a * 2 * D + 16 * ((d / 8) ^ v_sw<D>(key_a)) + (d % 8) * 2;
    }
  }

  vmem_drain();
  __syncthreads();
  dma_wait_barrier();
  for (int kb = 0; kb < nkb; ++kb) {
    if (AB < 4 && kb + 1 < nkb)
      stage_block<D>(kbase, vbase, smem + ((kb + 1) & 1) * C::STAGE, (kb + 1) * C::KB, S, wave, lane);
    const char* kl = smem + (AB >= 4 ? 0 : (kb & 1)) * C::STAGE;
    const char* vl = kl + C::K_BYTES;
    const bool two = (S - kb * C::KB) >= 64;   // the last block may hold a single 32-key tile
    if (active) {
      // ---------------- S^T = K Q^T for both tiles (independent int8 MFMA chains)
      v16i acc[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        v4i kf[C::NKS];
#pragma unroll
        for (int s = 0; s < C::NKS; ++s)
          kf[s] = *reinterpret_cast<const v4i*>(kl + koff[s] + u * 32 * D);
        if constexpr (AB == 3) {
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[u][i] = kf[i & 3][i >> 2] + qf[i & 3][0];
        } else {
          acc[u] = mfma_i8(kf[0], qf[0], v16i{});
#pragma unroll
          for (int s = 1; s < C::NKS; ++s) acc[u] = mfma_i8(kf[s], qf[s], acc[u]);
        }
      }
      v4u pw[2][2];
      if constexpr (AB == 1 || AB == 5) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int g = 0; g < 2; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j) pw[u][g][j] = (unsigned)acc[u][8 * g + 2 * j] & 0x3fff3fffu;
      } else {
      // ---------------- S = fp16(acc * sq*sk*qks), tile row maxima
      v2h s2[2][8];
      _Float16 rm[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float c = cq * (float)sk_lds[min(kb * 2 + u, S / 32 - 1)];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s2[u][j][0] = (_Float16)((float)acc[u][2 * j] * c);
          s2[u][j][1] = (_Float16)((float)acc[u][2 * j + 1] * c);
        }
        v2h mx = __builtin_elementwise_max(__builtin_elementwise_max(s2[u][0], s2[u][1]),
                                           __builtin_elementwise_max(s2[u][2], s2[u][3]));
        mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(
                                               __builtin_elementwise_max(s2[u][4], s2[u][5]),
                                               __builtin_elementwise_max(s2[u][6], s2[u][7])));
        rm[u] = (_Float16)pair_max(vmax((float)mx[0], (float)mx[1]));
      }
      if (!two) {  // a lone last tile: make tile 1 contribute exactly nothing
        rm[1] = rm[0];
#pragma unroll
        for (int j = 0; j < 8; ++j) s2[1][j] = v2h{(_Float16)-65504.0f, (_Float16)-65504.0f};
      }
      // deferred max shared by the two tiles (cdna_hip_programming.md T13): the running max moves
      // only when some row's tile max exceeds it by more than THR = 8 (log2 units).  P_i8 depends
      // only on S - rowmax(tile); O and l share the (possibly stale) reference, so O / l is the
      // same up to rounding, and the fp16 PV operands stay <= 2^8.
      const _Float16 rmb = rm[0] > rm[1] ? rm[0] : rm[1];
      const bool grow = __ballot((float)rmb > (float)m + 8.0f) != 0;
      float r = 1.0f;
      if (grow) {
        const _Float16 nm = m > rmb ? m : rmb;
        r = exp2_f32((float)(_Float16)(m - nm));
        m = nm;
      }
      // ---------------- e = exp2(S - rm), P_i8 = trunc(127 e), operand = P_i8 * sp (packed fp16)
      float lt = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float er = exp2_f32((float)(_Float16)(rm[u] - m));   // P = e * exp2(rm - m)
        const v2h rm2 = {rm[u], rm[u]};
        const _Float16 sp16 = (_Float16)(er * (1.0f / 127.0f));
        const v2h sp2 = {sp16, sp16};
        float esum = 0.f;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          v2h d2[4], e2[4], t2[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) d2[j] = s2[u][4 * g + j] - rm2;
          exp2_pk4(d2, e2);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            esum = __builtin_amdgcn_fdot2(e2[j], one2, esum, false);
            d2[j] = e2[j] * k127;
          }
          trunc_pk4(d2, t2);
#pragma unroll
          for (int j = 0; j < 4; ++j) pw[u][g][j] = __builtin_bit_cast(unsigned, t2[j] * sp2);
        }
        lt += esum * er;
      }
      l = l * r + pair_sum(lt);
      if (grow) {
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) o[b] *= r;
      }
      }
      // ---------------- O^T += Vdq^T P^T (fp16 MFMA, fp32 accumulate)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int b = 0; b < C::NDB; ++b) {
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const char* va = vl + voff[b] + (32 * u + 16 * s) * 2 * D;
            const v8h a = __builtin_bit_cast(v8h, ds_read_tr16_x2(va, va + 8 * 2 * D));
            if constexpr (AB == 2) {
              asm volatile("" :: "v"(a), "v"(pw[u][s]));
            } else {
              o[b] = mfma_f16(a, __builtin_bit_cast(v8h, pw[u][s]), o[b]);
            }
          }
        }
      }
    }
    if constexpr (AB < 4) dma_wait_barrier();
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
      for (int j = 0; j < 4; ++j) w[j] = (_Float16)(o[b][4 * g + j] * il);
      *reinterpret_cast<v4h*>(orow + 32 * b + 8 * g + 4 * h) = w;
    }
  }
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_int8_attn_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                                   const void* vdq, void* out, void* lse, long bh, long seq,
                                   int head_dim, float qks, void* stream) {
  if (seq % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0 || seq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
#define QA_LAUNCH(Dv)                                                                           \
  {                                                                                             \
    using C = Int8FwdCfg<Dv>;                                                                   \
    const int nq = (int)((seq + C::QROWS - 1) / C::QROWS);                                      \
    const int lds = 2 * C::STAGE + (int)(((seq / 32) * 2 + 15) / 16 * 16);                     \
    hipFuncSetAttribute((const void*)int8_attn_fwd_kernel<Dv>,                                  \
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds);                       \
    hipLaunchKernelGGL((int8_attn_fwd_kernel<Dv>), dim3((unsigned)(nq * bh)), dim3(64 * C::WAVES), lds, st, \
                       (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8,            \
                       (const _Float16*)sk, (const _Float16*)vdq, (_Float16*)out, (_Float16*)lse, \
                       (int)bh, (int)seq, qks);                                                 \
  }
  if (head_dim == 128) QA_LAUNCH(128) else QA_LAUNCH(64)
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_attn_fwd_ablate(const void* q_i8, const void* sq, const void* k_i8,
                                          const void* sk, const void* vdq, void* out, void* lse,
                                          long bh, long seq, float qks, int ab, void* stream) {
  using C = Int8FwdCfg<128>;
  const int nq = (int)((seq + C::QROWS - 1) / C::QROWS);
  const int lds = 2 * C::STAGE + (int)(((seq / 32) * 2 + 15) / 16 * 16);
  hipStream_t st = (hipStream_t)stream;
#define QA_AB(A)                                                                                  \
  hipFuncSetAttribute((const void*)int8_attn_fwd_kernel<128, A>,                                  \
                      hipFuncAttributeMaxDynamicSharedMemorySize, lds);                           \
  hipLaunchKernelGGL((int8_attn_fwd_kernel<128, A>), dim3((unsigned)(nq * bh)), dim3(64 * C::WAVES), \
                     lds, st, (const int8_t*)q_i8, (const _Float16*)sq, (const int8_t*)k_i8,       \
                     (const _Float16*)sk, (const _Float16*)vdq, (_Float16*)out, (_Float16*)lse,    \
                     (int)bh, (int)seq, qks);
  switch (ab) {
    case 1: QA_AB(1) break;
    case 2: QA_AB(2) break;
    case 3: QA_AB(3) break;
    case 4: QA_AB(4) break;
    case 5: QA_AB(5) break;
    default: QA_AB(0) break;
  }
#undef QA_AB
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
