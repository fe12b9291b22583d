// MX-FP4 attention forward for gfx950 inference (SageAttention3's FP4 path, which
// the reference names in README.md:49-55 but does not implement).  Everything below is defined
// here; oracle/restate.py mxfp4_fwd restates it and tests/test_gpu_mxfp4.py checks the kernels.
//
// Number format: OCP MX (v1.0) FP4 = e2m1 elements {0, ±0.5, ±1, ±1.5, ±2, ±3, ±4, ±6} sharing one
// power-of-two e8m0 scale per block of 32.  Block scale 2^e with e = floor(log2 amax) - 2 (amax = 0:
// e = -127); element = RNE(saturate(x / 2^e)) -- exactly v_cvt_scalef32_pk_fp4_f32.
//   Q, K: blocks of 32 along D per row  (the K dimension of S = Q K^T).
//   V   : blocks of 32 keys per column d (the K dimension of O = P V), stored transposed in operand
//         order: per 64-key tile g and column d, 2 x 16 bytes, half h holding the 32 keys
//         64g + 32(j>>4) + 8((j>>2)&3) + 4h + (j&3), j = 0..31 (nibble j, low nibble first) --
//         the key order in which a lane holds P after the swapped S^T = K Q^T product.
//   P   : per query row, one block per lane half: the 32 probabilities the lane holds of a 64-key
//         tile (same interleaved key set as V's block h), scale from their own max.
// Attention per 64-key tile: S = (deq Q)(deq K)^T exactly (block-scaled fp4 MFMA, fp32
// accumulation); m = ceil(rowmax(S * qks)) when that max exceeds the running m by more than 8
// (else m stays; m starts at -inf), O and l scaled by the exact power of two 2^(m_old - m_new);
// P = exp2(fma(S, qks, -m)) in fp32 (so P <= 2^8); P_fp4 = MX(P); l += sum(deq P_fp4);
// O += (deq P_fp4)(deq V).  Out: O / l (fp16), lse = m + log2(l) (fp32, base 2).  Because every
// rescale is a power of two, the fp4 codes of P do not depend on when m was raised.
#include "common.h"

namespace qattn {

typedef int v8i_t __attribute__((ext_vector_type(8)));

QA_DEVICE unsigned e8m0_of(float amax) {
  // floor(log2 amax) - 2 as a biased e8m0 byte (inputs are fp16, so amax is a normal fp32 or 0)
  if (!(amax > 0.f)) return 0u;
  const int e = (int)((__float_as_uint(amax) >> 23) & 0xff) - 127 - 2;
  return (unsigned)min(max(e + 127, 0), 254);
}
QA_DEVICE float e8m0_value(unsigned b) {
  return b == 0 ? 5.877471754111438e-39f : __uint_as_float(b << 23);   // 2^-127 is a denormal
}

// Pack 32 floats into 4 dwords of e2m1 (element j at nibble j, low nibble first) with scale s.
QA_DEVICE v4i pack_fp4x32(const float* x, float s) {
  v4i w;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    unsigned u = 0;
    u = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(u, x[8 * d + 0], x[8 * d + 1], s, 0);
    u = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(u, x[8 * d + 2], x[8 * d + 3], s, 1);
    u = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(u, x[8 * d + 4], x[8 * d + 5], s, 2);
    u = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(u, x[8 * d + 6], x[8 * d + 7], s, 3);
    w[d] = (int)u;
  }
  return w;
}

// ------------------------------------------------------------------------------ quantisers
// Q / K: one thread per 32-element block of a row.  x f16 [rows, D] -> q4 [rows, D/2], sc [rows, D/32].
// With ``mean`` (f16 [rows/seq, D], SageAttention smoothing) the row is first f16(x - mean[row/seq]).
template <int D>
__global__ __launch_bounds__(256) void mx_quant_rows_kernel(const _Float16* __restrict__ x,
                                                            const _Float16* __restrict__ mean,
                                                            uint8_t* __restrict__ q4,
                                                            uint8_t* __restrict__ sc, long nblk, long seq) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nblk) return;
  const v8h* src = reinterpret_cast<const v8h*>(x + i * 32);
  constexpr int NB = D / 32;
  const v8h* mu = mean ? reinterpret_cast<const v8h*>(mean + (i / NB / seq) * D + (i % NB) * 32) : nullptr;
  float f[32];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v8h v = src[c];
    if (mu) {
      const v8h w = mu[c];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (_Float16)((float)v[j] - (float)w[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[8 * c + j] = (float)v[j];
      amax = fmaxf(amax, fabsf(f[8 * c + j]));
    }
  }
  const unsigned e = e8m0_of(amax);
  reinterpret_cast<v4i*>(q4)[i] = pack_fp4x32(f, e8m0_value(e));
  sc[i] = (uint8_t)e;
}

// V: one thread per (head, 64-key tile g, column d, half h).  v f16 [BH*Sk, D] ->
// vt [BH][Sk/64][D][32 B] (operand order, see the header) and vs [BH][Sk/64][D][2].
template <int D>
__global__ __launch_bounds__(256) void mx_quant_vt_kernel(const _Float16* __restrict__ v,
                                                          uint8_t* __restrict__ vt,
                                                          uint8_t* __restrict__ vs, long nthr, int Sk) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nthr) return;
  const int h = (int)(i & 1);
  const int d = (int)((i >> 1) % D);
  const long gt = (i >> 1) / D;                 // head * (Sk/64) + g
  const int ng = Sk / 64;
  const long bh = gt / ng;
  const int g = (int)(gt % ng);
  const _Float16* col = v + ((long)bh * Sk + 64L * g) * D + d;
  float f[32];
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int key = 32 * (j >> 4) + 8 * ((j >> 2) & 3) + 4 * h + (j & 3);
    f[j] = (float)col[(long)key * D];
    amax = fmaxf(amax, fabsf(f[j]));
  }
  const unsigned e = e8m0_of(amax);
  reinterpret_cast<v4i*>(vt)[i] = pack_fp4x32(f, e8m0_value(e));
  vs[i] = (uint8_t)e;
}

// ------------------------------------------------------------------------------ attention
template <int D>
struct MxCfg {
  static constexpr int WAVES = 4;
  static constexpr int QROWS = 32 * WAVES;
  static constexpr int KT = 64;                       // keys per tile / ring slot
  static constexpr int NSLOT = 4;
  static constexpr int KROWB = D / 2;                 // fp4 bytes per key row
  static constexpr int K_BYTES = KT * KROWB;          // 4 KiB at D = 128
  static constexpr int V_BYTES = D * 32;              // [D][32 B]
  static constexpr int KS_BYTES = KT * (D / 32);      // key scales of the tile
  static constexpr int VS_BYTES = D * 2;
  static constexpr int KOFF = 0, VOFF = K_BYTES, KSOFF = K_BYTES + V_BYTES, VSOFF = KSOFF + 256;
  static constexpr int SLOT = VSOFF + 256;
  static constexpr int P16 = (K_BYTES + V_BYTES) / 1024;   // 1-KiB pieces
  static constexpr int IPW16 = P16 / WAVES;
  static constexpr int IPW = IPW16 + 2;               // + the two 256-B scale blocks
  static constexpr int NKS = D / 64;                  // 32x32x64 k-steps of S
  static constexpr int NDB = D / 32;
  static constexpr float MSLACK = 8.f;                // P <= 2^MSLACK between max raises
  static_assert(KS_BYTES <= 256 && VS_BYTES <= 256 && P16 % WAVES == 0, "tile layout");
};

#ifndef QA_MX_OCC
#define QA_MX_OCC 2   // min waves per SIMD the register budget is sized for
#endif
template <int D>
__global__ __launch_bounds__(256, QA_MX_OCC) void mxfp4_attn_fwd_kernel(
    const uint8_t* __restrict__ q4, const uint8_t* __restrict__ qs, const uint8_t* __restrict__ k4,
    const uint8_t* __restrict__ ks, const uint8_t* __restrict__ vt, const uint8_t* __restrict__ vs,
    _Float16* __restrict__ out, float* __restrict__ lse, int BH, int Sq, int Sk, int G, float qks) {
  using C = MxCfg<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nq = (Sq + C::QROWS - 1) / C::QROWS;
  int bh, qt;
  xcd_remap(blockIdx.x, nq, BH, bh, qt);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, h = lane >> 5, c32 = lane & 31;
  const int q0 = qt * C::QROWS + wave * 32;
  const bool active = q0 < Sq;
  const int qi = min(q0 + c32, Sq - 1);
  const long kvh = bh / G;
  const int nt = Sk / C::KT;

  // ---- LDS-DMA plan: pieces 0..P16-1 of (K | V^T) and one dma4 each for the two scale blocks
  const char* kbase = reinterpret_cast<const char*>(k4 + kvh * Sk * C::KROWB);
  const char* vbase = reinterpret_cast<const char*>(vt + kvh * (long)nt * C::V_BYTES);
  const char* ksbase = reinterpret_cast<const char*>(ks + kvh * Sk * (D / 32));
  const char* vsbase = reinterpret_cast<const char*>(vs + kvh * (long)nt * C::VS_BYTES);
  unsigned voff[C::IPW16], loff[C::IPW16], stride[C::IPW16];
  v4u rs[C::IPW16];
#pragma unroll
  for (int i = 0; i < C::IPW16; ++i) {
    const int p = wave + C::WAVES * i;
    const bool isv = p >= C::K_BYTES / 1024;
    const int piece = isv ? p - C::K_BYTES / 1024 : p;
    voff[i] = piece * 1024 + 16 * lane;
    loff[i] = (isv ? C::VOFF : C::KOFF) + piece * 1024;
    stride[i] = isv ? C::V_BYTES : C::K_BYTES;
    rs[i] = make_rsrc(isv ? vbase : kbase, (unsigned)(nt * (isv ? C::V_BYTES : C::K_BYTES)));
  }
  const v4u ks_rs = make_rsrc(ksbase, (unsigned)(nt * C::KS_BYTES));
  const v4u vs_rs = make_rsrc(vsbase, (unsigned)(nt * C::VS_BYTES));
  const unsigned smem_lds = lds_addr(smem);
  auto issue = [&](unsigned slot, int t) {
#pragma unroll
    for (int i = 0; i < C::IPW16; ++i) dma16_buf(rs[i], voff[i], (unsigned)t * stride[i], slot + loff[i]);
    dma4_buf(ks_rs, 4 * lane, (unsigned)t * C::KS_BYTES, slot + C::KSOFF);
    dma4_buf(vs_rs, 4 * lane, (unsigned)t * C::VS_BYTES, slot + C::VSOFF);
  };
#pragma unroll
  for (int i = 0; i < C::NSLOT - 1; ++i) issue(smem_lds + i * C::SLOT, min(i, nt - 1));

  // ---- own query fragments (B operand of S^T): lane holds Q[qi][64s + 32h .. +32] and its scales
  v4i qf[C::NKS];
  unsigned qsw;
  {
    const long r = (long)bh * Sq + qi;
#pragma unroll
    for (int s = 0; s < C::NKS; ++s) qf[s] = *reinterpret_cast<const v4i*>(q4 + r * C::KROWB + 32 * s + 16 * h);
    qsw = 0;
#pragma unroll
    for (int b = 0; b < D / 32; ++b) qsw |= (unsigned)qs[r * (D / 32) + b] << (8 * b);
  }

  v16f o[C::NDB];
#pragma unroll
  for (int b = 0; b < C::NDB; ++b) o[b] = v16f{};
  float m = -INFINITY, l = 0.f;   // integer running max (log2 units), sum of the quantised P

  vmem_drain();
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    ring_wait_barrier<2 * C::IPW>();   // tile t landed (t+1, t+2 may be in flight); slot (t+3)&3 is free
    issue(smem_lds + ((t + 3) & 3) * C::SLOT, min(t + 3, nt - 1));
    const char* sl = smem + (t & 3) * C::SLOT;
    // S^T for the two 32-key halves u: A = K rows 32u + c32, k = 64s + 32h .. +32
    v16f acc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      acc[u] = v16f{};
      const int key = 32 * u + c32;
      const unsigned ksw = *reinterpret_cast<const unsigned*>(sl + C::KSOFF + key * (D / 32));
#pragma unroll
      for (int s = 0; s < C::NKS; ++s) {
        const v4i ka = *reinterpret_cast<const v4i*>(sl + C::KOFF + key * C::KROWB + 32 * s + 16 * h);
        const v8i_t a = {ka[0], ka[1], ka[2], ka[3], 0, 0, 0, 0};
        const v8i_t b = {qf[s][0], qf[s][1], qf[s][2], qf[s][3], 0, 0, 0, 0};
        const int sa = (int)((ksw >> (8 * (2 * s + h))) & 0xff);
        const int sb = (int)((qsw >> (8 * (2 * s + h))) & 0xff);
        acc[u] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc[u], 4, 4, 0, sa, 0, sb);
      }
    }
    // online softmax over the tile (fp32); the lane holds 32 keys of its query row.  m is an
    // integer (log2 units) raised only when the row max exceeds it by more than MSLACK, so every
    // rescale is an exact power of two and, between raises, P <= 2^MSLACK needs no rescale at all.
    float amx = acc[0][0];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = (u == 0 ? 1 : 0); r < 16; ++r) amx = fmaxf(amx, acc[u][r]);
    const float lmx = amx * qks;                                  // this lane's max of S * qks
    const float mx = fmaxf(lmx, xor32_swap(lmx, lane));
    if (__ballot(mx > m + C::MSLACK)) {
      const float nm = mx > m + C::MSLACK ? ceilf(mx) : m;
      const float rsc = m == -INFINITY ? 0.f : __builtin_ldexpf(1.f, (int)(m - nm));
      m = nm;
      l *= rsc;
#pragma unroll
      for (int b = 0; b < C::NDB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[b][i] = o[b][i] * rsc;
    }
    const float nm = -m;
    float x[32];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) x[16 * u + r] = exp2_f32(__builtin_fmaf(acc[u][r], qks, nm));
    // the block max is exp2 of the lane's max argument (exp2 and the fma are monotonic)
    const float pmax = exp2_f32(__builtin_fmaf(amx, qks, nm));
    // P block of this lane half: its 32 values, nibble j = 16u + r
    const unsigned pe = e8m0_of(pmax);
    const v4i pk = pack_fp4x32(x, e8m0_value(pe));
    const v8i_t pb = {pk[0], pk[1], pk[2], pk[3], 0, 0, 0, 0};
    // row sum of the quantised P on the matrix core: every row of ONES . P^T is the column sum
    {
      const v8i_t ones = {0x22222222, 0x22222222, 0x22222222, 0x22222222, 0, 0, 0, 0};   // e2m1 1.0
      const v16f ts = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ones, pb, v16f{}, 4, 4, 0, 127, 0,
                                                                      (int)pe);
      l += ts[0];
    }
    // O^T[d][q] += V^T[d][keys] P^T[keys][q], A = V^T rows d = 32b + c32, k = the half-h key set
#pragma unroll
    for (int b = 0; b < C::NDB; ++b) {
      const int d = 32 * b + c32;
      const v4i va = *reinterpret_cast<const v4i*>(sl + C::VOFF + d * 32 + 16 * h);
      const v8i_t a = {va[0], va[1], va[2], va[3], 0, 0, 0, 0};
      const int sa = (int)*reinterpret_cast<const uint8_t*>(sl + C::VSOFF + 2 * d + h);
      o[b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, pb, o[b], 4, 4, 0, sa, 0, (int)pe);
    }
  }
  vmcnt_wait_all();
  __syncthreads();
  if (!active) return;
  const long row0 = (long)bh * Sq + q0;
  if (h == 0) lse[row0 + c32] = m + log2_f32(l);
  static_assert(C::WAVES * RowTile<D, _Float16>::BYTES <= C::NSLOT * C::SLOT, "staging fits the ring");
  store_rows<D, _Float16>(o, 1.0f / l, smem + wave * RowTile<D, _Float16>::BYTES, out + row0 * D, lane);
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_mxfp4_quant_rows(const void* x, const void* mean, void* q4, void* scale, long rows,
                                      long seq, int head_dim, void* stream) {
  if (head_dim != 64 && head_dim != 128) return 1;
  if (mean && (seq <= 0 || rows % seq != 0)) return 1;
  const long nblk = rows * head_dim / 32;
  if (nblk == 0) return 0;
  dim3 grid((unsigned)((nblk + 255) / 256)), block(256);
  if (head_dim == 128)
    hipLaunchKernelGGL((mx_quant_rows_kernel<128>), grid, block, 0, (hipStream_t)stream,
                       (const _Float16*)x, (const _Float16*)mean, (uint8_t*)q4, (uint8_t*)scale, nblk, seq);
  else
    hipLaunchKernelGGL((mx_quant_rows_kernel<64>), grid, block, 0, (hipStream_t)stream,
                       (const _Float16*)x, (const _Float16*)mean, (uint8_t*)q4, (uint8_t*)scale, nblk, seq);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_mxfp4_quant_vt(const void* v, void* vt, void* vscale, long bh, long seq, int head_dim,
                                    void* stream) {
  if (seq % 64 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  const long nthr = bh * (seq / 64) * head_dim * 2;
  if (nthr == 0) return 0;
  dim3 grid((unsigned)((nthr + 255) / 256)), block(256);
  if (head_dim == 128)
    hipLaunchKernelGGL((mx_quant_vt_kernel<128>), grid, block, 0, (hipStream_t)stream,
                       (const _Float16*)v, (uint8_t*)vt, (uint8_t*)vscale, nthr, (int)seq);
  else
    hipLaunchKernelGGL((mx_quant_vt_kernel<64>), grid, block, 0, (hipStream_t)stream,
                       (const _Float16*)v, (uint8_t*)vt, (uint8_t*)vscale, nthr, (int)seq);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_mxfp4_attn_fwd(const void* q4, const void* qscale, const void* k4,
                                    const void* kscale, const void* vt, const void* vscale, void* out,
                                    void* lse, long bh, long sq, long sk, int group, int head_dim,
                                    float qks, void* stream) {
  if (sq % 32 != 0 || sk % 64 != 0 || group < 1 || bh % group != 0 || head_dim != 128) return 1;
  if (bh == 0 || sq == 0) return 0;
  if (sk == 0) return 1;
  using C = MxCfg<128>;
  const int nq = (int)((sq + C::QROWS - 1) / C::QROWS);
  const int lds = C::NSLOT * C::SLOT;
  { static LdsGrant granted_; lds_grant((const void*)mxfp4_attn_fwd_kernel<128>, lds, granted_); }
  hipLaunchKernelGGL((mxfp4_attn_fwd_kernel<128>), dim3((unsigned)(nq * bh)), dim3(256), lds,
                     (hipStream_t)stream, (const uint8_t*)q4, (const uint8_t*)qscale, (const uint8_t*)k4,
                     (const uint8_t*)kscale, (const uint8_t*)vt, (const uint8_t*)vscale, (_Float16*)out,
                     (float*)lse, (int)bh, (int)sq, (int)sk, group, qks);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
