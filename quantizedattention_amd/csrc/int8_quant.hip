// SageAttention-3 per-block int8 quantiser (replaces the quantisation inside
// helion_atten_int8_hl_dot_fwd, attention_int8.py:178-195 and 241-247) and the k-smoothing mean
// (build contract for attention_int8.py:24-25).
//
// Numerics (bit-exact with the eager reference):
//   s   = RNE_fp16( fp32(amax|X|) / 127 )            (IEEE fp32 divide, once per block)
//   idx = trunc( RNE_fp16( fp32(x) / fp32(s) ) )      (fp16 round, then trunc; the division as a
//                                                       reciprocal and one Newton step, exactly:
//                                                       common.h quant_div)
// An all-zero block (s == 0) yields idx 0.
//
// HBM-bound: one wave per 32-token block (32 x D fp16 = 8 KB for D=128), 16-byte loads/stores,
// fully coalesced (1 KiB per wave instruction in, 512 B out).
#include "common.h"

namespace qattn {

// workgroups per head of the fused k-mean + k quantiser (A/B: 1 55.1-55.4 us, 2 71-72, 4 107-109 at
// config 3 against 54.5 us for qattn_kmean + qattn_int8_quant_img; HISTORY.md round 6)
#ifndef QA_KQ_SPLITS
#define QA_KQ_SPLITS 1
#endif

// max |x| over 8 fp16 values folded into a running pair of u16 maxima: for finite halves the order of
// |x| is the integer order of (bits & 0x7fff), so one v_and + one v_pk_max_u16 per pair (the f32 form
// takes a conversion and a max per value).  amax_pk_f32 turns the pair into the float max.
typedef unsigned short v2us __attribute__((ext_vector_type(2)));
QA_DEVICE void amax_pk8(const v8h& x, v2us& acc) {
  const v4u w = __builtin_bit_cast(v4u, x);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    acc = __builtin_elementwise_max(acc, __builtin_bit_cast(v2us, w[k] & 0x7fff7fffu));
}
QA_DEVICE float amax_pk_f32(v2us acc) {
  const unsigned short m = acc[0] > acc[1] ? acc[0] : acc[1];
  return (float)__builtin_bit_cast(_Float16, m);
}

// rows: total rows (multiple of 32); rows_per_head: S (for the k-mean lookup)
// DEQ: also write f16(idx * s) (the forward's P.V operand for v); IMG: also write bf16(idx) (the
// exact transposed-read image the backward's accumulating products use for q and k).
// km: the block's head mean row (SMOOTH; global or LDS memory)
template <int D, bool DEQ, bool SMOOTH, bool IMG>
QA_DEVICE void quant_block32(const _Float16* __restrict__ x, int8_t* __restrict__ idx,
                             _Float16* __restrict__ scale, _Float16* __restrict__ deq,
                             __bf16* __restrict__ img, const _Float16* km, long blk, int lane) {
  constexpr int ELEMS = 32 * D;        // elements per block
  constexpr int ITERS = ELEMS / 512;   // 8 halfs per lane per iteration
  const _Float16* xb = x + blk * ELEMS;
  v8h v[ITERS];
  v2us am = {0, 0};
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int e = (i * 64 + lane) * 8;
    v[i] = *reinterpret_cast<const v8h*>(xb + e);
    if constexpr (SMOOTH) {
      // f16(x - m) (eager fp16 `k - k_mean`): packed f16 subtraction, which rounds the exact
      // difference once -- the same bits as rounding through fp32 first, since an fp32 difference
      // of two fp16 values is inexact only when their exponents are more than 13 apart, and then
      // both roundings return the larger operand
      const int d0 = e % D;
      const v8h m = *reinterpret_cast<const v8h*>(km + d0);
      v2h xs[4], ms[4];
      __builtin_memcpy(xs, &v[i], 16);
      __builtin_memcpy(ms, &m, 16);
#pragma unroll
      for (int k = 0; k < 4; ++k) xs[k] = xs[k] - ms[k];   // v_pk_add_f16 (neg)
      __builtin_memcpy(&v[i], xs, 16);
    }
    amax_pk8(v[i], am);
  }
  const float amax = wave_max_f(amax_pk_f32(am));
  const _Float16 s16 = (_Float16)(amax / 127.0f);
  const float s = (float)s16;
  const float r = quant_rcp(s);
  if (lane == 0) scale[blk] = s16;
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int e = (i * 64 + lane) * 8;
    unsigned lo, hi;
    v8h dq;
    float qf[8];
    quant8(v[i], s, r, lo, hi, qf);
    if constexpr (DEQ) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dq[j] = (_Float16)(qf[j] * s);
    }
    *reinterpret_cast<v2u*>(idx + blk * ELEMS + e) = v2u{lo, hi};
    if constexpr (DEQ) *reinterpret_cast<v8h*>(deq + blk * ELEMS + e) = dq;
    if constexpr (IMG) {
      const v4u w = {pk_bf16(qf[0], qf[1]), pk_bf16(qf[2], qf[3]), pk_bf16(qf[4], qf[5]),
                     pk_bf16(qf[6], qf[7])};
      *reinterpret_cast<v4u*>(img + blk * ELEMS + e) = w;
    }
  }
}
template <int D, bool DEQ, bool SMOOTH, bool IMG>
__global__ __launch_bounds__(256) void quant_block32_kernel(
    const _Float16* __restrict__ x, int8_t* __restrict__ idx, _Float16* __restrict__ scale,
    _Float16* __restrict__ deq, __bf16* __restrict__ img, const _Float16* __restrict__ kmean,
    long nblocks, int rows_per_head) {
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblocks) return;
  const _Float16* km = SMOOTH ? kmean + (blk * 32 / rows_per_head) * D : nullptr;
  quant_block32<D, DEQ, SMOOTH, IMG>(x, idx, scale, deq, img, km, blk, threadIdx.x & 63);
}

// ------------------------------------------------------------ V with the int8 P.V operand image
// One wave per 32-row block of v: the reference quantiser (v_i8 row-major + sv, bit-exact as above)
// and, of the same indices, the V^T operand image vt of the forward's int8 P.V product
// (qattn_int8_attn_fwd_ex): per block D/32 pieces of 1 KiB; piece b holds for lane
// L = 32h + c the 16 bytes v_i8[key pi(h, j)][32b + c], j = 0..15, pi(h, j) = (j & 3) + 8(j >> 2) + 4h
// -- the A operand of v_mfma_i32_32x32x32_i8 for V^T in the key order of the S^T accumulator
// (common.h).  Lane (row c, half h) loads v[c][32b + 16h .. +16]: exactly the A operand of the
// block in natural order, which one i8 MFMA against the identity transposes into that image.
template <int D>
QA_DEVICE void quant_vt(const _Float16* __restrict__ v, int8_t* __restrict__ vi,
                        _Float16* __restrict__ sv, int8_t* __restrict__ vt, long blk, int lane) {
  constexpr int NDB = D / 32;
  const int h = lane >> 5, c = lane & 31;
  const long row = blk * 32 + c;
  v8h x[NDB][2];
  v2us am = {0, 0};
#pragma unroll
  for (int b = 0; b < NDB; ++b)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      x[b][u] = *reinterpret_cast<const v8h*>(v + row * D + 32 * b + 16 * h + 8 * u);
      amax_pk8(x[b][u], am);
    }
  const float amax = wave_max_f(amax_pk_f32(am));
  const _Float16 s16 = (_Float16)(amax / 127.0f);
  const float s = (float)s16;
  const float r = quant_rcp(s);
  if (lane == 0) sv[blk] = s16;
  const v4i ident = identity_b_i8(lane);
#pragma unroll
  for (int b = 0; b < NDB; ++b) {
    unsigned w[4];
    float qf[8];
    quant8(x[b][0], s, r, w[0], w[1], qf);
    quant8(x[b][1], s, r, w[2], w[3], qf);
    const v4i a = {(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
    *reinterpret_cast<v4i*>(vi + row * D + 32 * b + 16 * h) = a;
    const v16i t = mfma_i8(a, ident, v16i{});
    *reinterpret_cast<v4i*>(vt + blk * 32 * D + b * 1024 + 16 * lane) = pack_acc_bytes(t);
  }
}
template <int D>
__global__ __launch_bounds__(256) void quant_vt_kernel(const _Float16* __restrict__ v,
                                                       int8_t* __restrict__ vi,
                                                       _Float16* __restrict__ sv,
                                                       int8_t* __restrict__ vt, long nblocks) {
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblocks) return;
  quant_vt<D>(v, vi, sv, vt, blk, threadIdx.x & 63);
}
// vt from stored indices (an int8 key/value cache restored from its wire format, kv_cache.py)
template <int D>
__global__ __launch_bounds__(256) void v_image_kernel(const int8_t* __restrict__ vi,
                                                      int8_t* __restrict__ vt, long nblocks) {
  constexpr int NDB = D / 32;
  const int lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31;
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblocks) return;
  const long row = blk * 32 + c;
  const v4i ident = identity_b_i8(lane);
#pragma unroll
  for (int b = 0; b < NDB; ++b) {
    const v4i a = *reinterpret_cast<const v4i*>(vi + row * D + 32 * b + 16 * h);
    const v16i t = mfma_i8(a, ident, v16i{});
    *reinterpret_cast<v4i*>(vt + blk * 32 * D + b * 1024 + 16 * lane) = pack_acc_bytes(t);
  }
}

// k_mean[bh][d] = fp16( sum_s fp32(k[bh][s][d]) / S )   (eager `k.mean(-2)` in fp16, fp32 accumulate)
// One 1024-thread workgroup per head; 4 independent 16-B loads in flight per thread.
template <int D>
__global__ __launch_bounds__(1024) void kmean_kernel(const _Float16* __restrict__ k,
                                                     _Float16* __restrict__ kmean, int S) {
  constexpr int TPR = D / 8;           // threads per row (8 halfs each)
  constexpr int RPI = 1024 / TPR;      // rows per step
  constexpr int U = 4;                 // steps unrolled
  __shared__ float part[RPI][D + 1];
  const int bh = blockIdx.x;
  const int t = threadIdx.x;
  const int c = (t % TPR) * 8, r0 = t / TPR;
  const _Float16* kb = k + (long)bh * S * D;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int r = r0;
  for (; r + (U - 1) * RPI < S; r += U * RPI) {
    v8h x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = *reinterpret_cast<const v8h*>(kb + (long)(r + u * RPI) * D + c);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)x[u][j];
  }
  for (; r < S; r += RPI) {
    const v8h x = *reinterpret_cast<const v8h*>(kb + (long)r * D + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (float)x[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[r0][c + j] = acc[j];
  __syncthreads();
  if (t < D) {
    float sum = 0.f;
    for (int i = 0; i < RPI; ++i) sum += part[i][t];
    kmean[(long)bh * D + t] = (_Float16)(sum / (float)S);
  }
}

// k-mean and the smoothed k quantiser in one launch (the two passes of qattn_kmean +
// qattn_int8_quant_img with kmean): SPLITS 1024-thread workgroups per head each sum the whole head
// (kmean_kernel's arithmetic and order, so k_mean is bit-identical; the repeated reads of a head
// hit the L2 / Infinity Cache), keep the mean in LDS, and quantise their 1/SPLITS of the head's
// 32-row blocks from the cache with it.  Split 0 writes k_mean.
template <int D, bool IMG, int SPLITS>
__global__ __launch_bounds__(1024) void kmean_quant_kernel(const _Float16* __restrict__ k,
                                                           _Float16* __restrict__ kmean,
                                                           int8_t* __restrict__ idx,
                                                           _Float16* __restrict__ scale,
                                                           __bf16* __restrict__ img, int S) {
  constexpr int TPR = D / 8;
  constexpr int RPI = 1024 / TPR;
  constexpr int U = 4;
  __shared__ float part[RPI][D + 1];
  __shared__ __attribute__((aligned(16))) _Float16 km[D];
  const int bh = blockIdx.x / SPLITS, sp = blockIdx.x % SPLITS;
  const int t = threadIdx.x;
  const int c = (t % TPR) * 8, r0 = t / TPR;
  const _Float16* kb = k + (long)bh * S * D;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int r = r0;
  for (; r + (U - 1) * RPI < S; r += U * RPI) {
    v8h x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = *reinterpret_cast<const v8h*>(kb + (long)(r + u * RPI) * D + c);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)x[u][j];
  }
  for (; r < S; r += RPI) {
    const v8h x = *reinterpret_cast<const v8h*>(kb + (long)r * D + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (float)x[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[r0][c + j] = acc[j];
  __syncthreads();
  if (t < D) {
    float sum = 0.f;
    for (int i = 0; i < RPI; ++i) sum += part[i][t];
    const _Float16 m = (_Float16)(sum / (float)S);
    km[t] = m;
    if (sp == 0) kmean[(long)bh * D + t] = m;
  }
  __syncthreads();
  const int nb = S / 32, per = (nb + SPLITS - 1) / SPLITS;
  const int b1 = min(nb, (sp + 1) * per);
  for (int b = sp * per + (t >> 6); b < b1; b += 16)
    quant_block32<D, false, true, IMG>(k, idx, scale, nullptr, img, km, (long)bh * nb + b, t & 63);
}

}  // namespace qattn

using namespace qattn;

extern "C" int qattn_int8_quant_k_smooth(const void* k, void* kmean, void* k_i8, void* sk, void* k_bf,
                                         long bh, long seq, int head_dim, void* stream) {
  if (seq % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (bh == 0 || seq == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  constexpr int SP = QA_KQ_SPLITS;
  const dim3 grid((unsigned)(bh * SP)), block(1024);
#define QA_LAUNCH(Dv, IM)                                                                              \
  hipLaunchKernelGGL((kmean_quant_kernel<Dv, IM, SP>), grid, block, 0, st, (const _Float16*)k,        \
                     (_Float16*)kmean, (int8_t*)k_i8, (_Float16*)sk, (__bf16*)k_bf, (int)seq)
  if (head_dim == 128) {
    if (k_bf) QA_LAUNCH(128, true); else QA_LAUNCH(128, false);
  } else {
    if (k_bf) QA_LAUNCH(64, true); else QA_LAUNCH(64, false);
  }
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_quant_img(const void* x, void* idx, void* scale, void* deq, void* img,
                                    const void* kmean, long rows, int rows_per_head, int head_dim,
                                    void* stream) {
  if (rows % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  if (kmean && rows_per_head % 32 != 0) return 1;
  const long nblocks = rows / 32;
  if (nblocks == 0) return 0;
  dim3 grid((unsigned)((nblocks + 3) / 4)), block(256);
  hipStream_t st = (hipStream_t)stream;
  auto X = (const _Float16*)x;
  auto I = (int8_t*)idx;
  auto Sc = (_Float16*)scale;
  auto Q = (_Float16*)deq;
  auto B = (__bf16*)img;
  auto M = (const _Float16*)kmean;
#define QA_LAUNCH(Dv, DQ, SM, IM)                                                                    \
  hipLaunchKernelGGL((quant_block32_kernel<Dv, DQ, SM, IM>), grid, block, 0, st, X, I, Sc, Q, B, M, \
                     nblocks, rows_per_head)
#define QA_LAUNCH_D(Dv)                                                                             \
  if (deq) {                                                                                        \
    if (kmean) QA_LAUNCH(Dv, true, true, false); else QA_LAUNCH(Dv, true, false, false);            \
  } else if (img) {                                                                                 \
    if (kmean) QA_LAUNCH(Dv, false, true, true); else QA_LAUNCH(Dv, false, false, true);            \
  } else {                                                                                          \
    if (kmean) QA_LAUNCH(Dv, false, true, false); else QA_LAUNCH(Dv, false, false, false);          \
  }
  if (deq && img) return 1;   // one extra output per launch
  if (head_dim == 128) { QA_LAUNCH_D(128) } else { QA_LAUNCH_D(64) }
#undef QA_LAUNCH_D
#undef QA_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_quant(const void* x, void* idx, void* scale, void* deq, const void* kmean,
                                long rows, int rows_per_head, int head_dim, void* stream) {
  return qattn_int8_quant_img(x, idx, scale, deq, nullptr, kmean, rows, rows_per_head, head_dim,
                              stream);
}

extern "C" int qattn_int8_quant_vt(const void* v, void* v_i8, void* sv, void* vt, long rows,
                                   int head_dim, void* stream) {
  if (rows % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  const long nblocks = rows / 32;
  if (nblocks == 0) return 0;
  dim3 grid((unsigned)((nblocks + 3) / 4)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL(quant_vt_kernel<128>, grid, block, 0, st, (const _Float16*)v, (int8_t*)v_i8,
                       (_Float16*)sv, (int8_t*)vt, nblocks);
  else
    hipLaunchKernelGGL(quant_vt_kernel<64>, grid, block, 0, st, (const _Float16*)v, (int8_t*)v_i8,
                       (_Float16*)sv, (int8_t*)vt, nblocks);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_int8_v_image(const void* v_i8, void* vt, long rows, int head_dim, void* stream) {
  if (rows % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  const long nblocks = rows / 32;
  if (nblocks == 0) return 0;
  dim3 grid((unsigned)((nblocks + 3) / 4)), block(256);
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL(v_image_kernel<128>, grid, block, 0, st, (const int8_t*)v_i8, (int8_t*)vt, nblocks);
  else
    hipLaunchKernelGGL(v_image_kernel<64>, grid, block, 0, st, (const int8_t*)v_i8, (int8_t*)vt, nblocks);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int qattn_kmean(const void* k, void* kmean, long bh, long seq, int head_dim, void* stream) {
  if (head_dim != 64 && head_dim != 128) return 1;
  if (bh == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (head_dim == 128)
    hipLaunchKernelGGL((kmean_kernel<128>), dim3((unsigned)bh), dim3(1024), 0, st, (const _Float16*)k,
                       (_Float16*)kmean, (int)seq);
  else
    hipLaunchKernelGGL((kmean_kernel<64>), dim3((unsigned)bh), dim3(1024), 0, st, (const _Float16*)k,
                       (_Float16*)kmean, (int)seq);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ------------------------------------------------------------------------- dequantised image
// deq = f16(idx * s) per 32-row block, exactly the DEQ output of the quantiser: rebuilds the P.V
// operand of a key/value cache restored from its int8 wire format (kv_cache.py).
// 8 elements per thread.
__global__ __launch_bounds__(256) void int8_dequant_kernel(const int8_t* __restrict__ idx,
                                                           const _Float16* __restrict__ scale,
                                                           _Float16* __restrict__ deq, long n8,
                                                           int block_elems) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  const float s = (float)scale[(i * 8) / block_elems];
  const v2u w = reinterpret_cast<const v2u*>(idx)[i];
  v8h o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int q = (int)(signed char)((w[j >> 2] >> (8 * (j & 3))) & 0xff);
    o[j] = (_Float16)((float)q * s);
  }
  reinterpret_cast<v8h*>(deq)[i] = o;
}

extern "C" int qattn_int8_dequant(const void* idx, const void* scale, void* deq, long rows,
                                  int head_dim, void* stream) {
  if (rows % 32 != 0 || (head_dim != 64 && head_dim != 128)) return 1;
  const long n8 = rows * head_dim / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(int8_dequant_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const int8_t*)idx, (const _Float16*)scale, (_Float16*)deq,
                     n8, 32 * head_dim);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
