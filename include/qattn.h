/*
 * qattn.h — C ABI of libqattn.so, the MI355X (gfx950) hot path of selau642/QuantizedAttention.
 *
 * The reference (three Python modules over Helion/Triton kernels) has no native boundary of its
 * own: each entry point below replaces one @helion.kernel call (or the torch glue around it) and is
 * cited as reference `file:line`.  The Python mirror of the reference's public functions
 * (quantizedattention_amd/attention_{int8,bf16,jvp}.py) binds exactly these symbols through ctypes
 * (quantizedattention_amd/_lib.py); INTEGRATION.md shows the binding for other hosts.
 *
 * Conventions (all entries):
 *   - Plain device pointers (HBM, allocated by the caller, contiguous row-major), sizes as long/int,
 *     `stream` is a hipStream_t (NULL = the default stream).  Work is enqueued asynchronously on
 *     `stream`; nothing is synchronised and no memory is allocated by the library.
 *   - Return value: 0 = enqueued, 1 = unsupported shape / argument (nothing launched),
 *     2 = launch failure (hipGetLastError() != hipSuccess).
 *   - "rows" N = BH * S with BH = batch * heads; tensors [B,H,S,D] are addressed as [BH*S, D].
 *     Block-scale arrays hold one fp16 per 32 consecutive rows: index (b*H+h)*S/32 + s/32
 *     (attention_int8.py:161-168).
 *   - qks = fp32(1/sqrt(D) * 1.44269504) (attention_int8.py:151-153, attention_bf16.py:188-190);
 *     sms = fp32(1/sqrt(D)).  lse values are base-2 (log2 of the softmax denominator plus max).
 *   - head_dim D in {64, 128}.  Dtypes: i8 = int8_t, f16 = _Float16 (IEEE half), bf16 = bfloat16,
 *     f32 = float.
 */
#ifndef QATTN_H
#define QATTN_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- versioning
 * QATTN_ABI_VERSION counts incompatible changes of the entries below (a changed argument list under
 * an old name; INTEGRATION.md §"ABI versions" lists them).  A host compiled against this header
 * checks qattn_abi_version() == QATTN_ABI_VERSION after loading the library and refuses to call it
 * otherwise: a library of another version would read its arguments with another meaning.
 * qattn_source_hash() is the sha256 (hex) of the kernel sources and compile flags the library was
 * built from (quantizedattention_amd/_srchash.py); the Python binding refuses a library whose hash
 * differs from the sources beside it (a stale prebuilt library). */
#define QATTN_ABI_VERSION 6
int qattn_abi_version(void);
const char* qattn_source_hash(void);

/* ---------------------------------------------------------------- int8 path (attention_int8.py) */

/* Per-32-row block quantiser (attention_int8.py:178-186 q, 188-195 k, 241-247 v).
 *   x      f16 [rows, D]              in
 *   idx    i8  [rows, D]              out: trunc(RNE_f16(f32(x') / f32(s)))
 *   scale  f16 [rows/32]              out: s = RNE_f16(amax|x'| / 127)   (all-zero block: s = 0, idx 0)
 *   deq    f16 [rows, D] or NULL      out: f16(idx * s)  (the fp16 operand of the forward P.V product)
 *   kmean  f16 [rows/rows_per_head, D] or NULL: when given, x' = f16(x - kmean[head]) (k-smoothing,
 *          build contract for attention_int8.py:24-25), else x' = x.
 * Bit-exact with the reference's eager-torch rounding.  rows % 32 == 0. */
int qattn_int8_quant(const void* x, void* idx, void* scale, void* deq, const void* kmean, long rows,
                     int rows_per_head, int head_dim, void* stream);
/* Same, with an optional exact bf16 image of idx (img bf16 [rows, D], or NULL): the backward's
 * transposed-read operand for q and k, written in the same pass.  deq and img are exclusive. */
int qattn_int8_quant_img(const void* x, void* idx, void* scale, void* deq, void* img,
                         const void* kmean, long rows, int rows_per_head, int head_dim,
                         void* stream);

/* deq = f16(idx * s) with s the block scale of each 32-row block (rows % 32 == 0): the quantiser's
 * deq output rebuilt from stored indices and scales (the int8 key/value cache of kv_cache.py). */
int qattn_int8_dequant(const void* idx, const void* scale, void* deq, long rows, int head_dim,
                       void* stream);

/* V quantiser for the int8 P.V product (attention_int8.py:241-247, same indices and scales as
 * qattn_int8_quant) that also writes the V^T operand image of those indices:
 *   v f16 [rows, D] -> v_i8 i8 [rows, D], sv f16 [rows/32] (bit-exact, as qattn_int8_quant) and
 *   vt i8 [rows/32][D/32][64][16]: for each 32-row block and 32-wide d block b, lane L = 32h + c holds
 *   v_i8[row pi(h, j)][32b + c], j = 0..15, pi(h, j) = (j & 3) + 8(j >> 2) + 4h (the A operand of
 *   v_mfma_i32_32x32x32_i8 in the forward's key order).  rows % 32 == 0. */
int qattn_int8_quant_vt(const void* v, void* v_i8, void* sv, void* vt, long rows, int head_dim,
                        void* stream);
/* vt of qattn_int8_quant_vt from stored indices v_i8 (a restored int8 key/value cache). */
int qattn_int8_v_image(const void* v_i8, void* vt, long rows, int head_dim, void* stream);

/* k_mean = f16(mean over the S tokens of each head) — k f16 [bh*seq, D] -> kmean f16 [bh, D]
 * (SageAttention smoothing; replaces the crashing `k.mean(0)` of attention_int8.py:24-25). */
int qattn_kmean(const void* k, void* kmean, long bh, long seq, int head_dim, void* stream);

/* qattn_kmean followed by qattn_int8_quant_img of the smoothed k, in one launch (attention_int8.py:
 * 24-25 smoothing, 188-195 k quantiser): kmean f16 [bh, D], k_i8 i8 [bh*seq, D], sk f16
 * [bh*seq/32] and (k_bf != NULL) the bf16 image bf16(k_i8) out, bit-identical with the two calls.
 * seq % 32 == 0. */
int qattn_int8_quant_k_smooth(const void* k, void* kmean, void* k_i8, void* sk, void* k_bf, long bh,
                              long seq, int head_dim, void* stream);

/* int8 SageAttention-3 forward, per (batch, head) (attention_int8.py:197-257; per-head contract F2).
 *   q_i8, k_i8  i8 [bh*seq, D]; sq, sk, sv f16 [bh*seq/32]; vt = the V^T operand image of
 *   qattn_int8_quant_vt; out O f16 [bh*seq, D]; lse f16 [bh*seq] (base 2).
 *   S = f16(f32(q_i8.k_i8) * sq*sk*qks), P = exp2(S - m), P_i8 = trunc(P / sp) with sp =
 *   exp2(rowmax - m)/127, and the P.V contraction on the int8 MFMA as the reference's
 *   hl.dot(P_int8, v_int8) (int8:249): each 32-key tile's exact int32 product is dequantised by
 *   sp * sv (int8:249-250).  seq % 32 == 0. */
int qattn_int8_attn_fwd(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                        const void* vt, const void* sv, void* out, void* lse, long bh, long seq,
                        int head_dim, float qks, void* stream);

/* Generalised shapes (the reference's int8 path has none of these): bh = batch *
 * query heads with sq_tok query rows each; the key/value tensors have bh / group heads of sk_tok
 * rows (query head h reads key/value head h / group: grouped-query attention); causal = 1 keeps
 * key <= query (top-left aligned positions), causal = 2 keeps key <= query + sk_tok - sq_tok
 * (bottom-right aligned: new queries against a key/value cache, sk_tok >= sq_tok); masked scores
 * are excluded.  Block scales index the
 * query rows and the key/value rows separately.  sq_tok % 32 == sk_tok % 32 == 0, bh % group == 0.
 * qattn_int8_attn_fwd is this with sq_tok = sk_tok = seq, group = 1, causal = 0.
 * The forward marks the (rare) waves whose literal-P-chain vote still holds at the end and redoes
 * them: qattn_int8_attn_fwd_qf in the same kernel, the entries on pre-quantised q
 * (and the split entry) with a second kernel on `stream`. */
int qattn_int8_attn_fwd_ex(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                           const void* vt, const void* sv, void* out, void* lse, long bh,
                           long sq_tok, long sk_tok, int group, int causal, int head_dim,
                           float qks, void* stream);

/* qattn_int8_attn_fwd_ex quantising q inside the attention kernel (the reference quantises inside its
 * forward, attention_int8.py:178-186): q f16 [bh*sq_tok, D] in; q_i8 i8 [bh*sq_tok, D] and sq f16
 * [bh*sq_tok/32] out, bit-exact with qattn_int8_quant; q_bf bf16 [bh*sq_tok, D] = bf16(q_i8) out
 * (the backward's image) when not NULL.  O and lse as qattn_int8_attn_fwd_ex on those q_i8, sq. */
int qattn_int8_attn_fwd_qf(const void* q, void* q_i8, void* sq, void* q_bf, const void* k_i8,
                           const void* sk, const void* vt, const void* sv, void* out, void* lse,
                           long bh, long sq_tok, long sk_tok, int group, int causal, int head_dim,
                           float qks, void* stream);

/* Key-split (flash-decoding) form of qattn_int8_attn_fwd_ex, non-causal, for short query blocks
 * against long key ranges (the int8 key/value cache): each workgroup covers
 * keys_per_split keys (multiple of 32) of its query rows and writes the partial softmax state
 *   opart f16 [nsplit][bh*sq_tok][D] = O_s / l_s (the key range's normalised output) and
 *   ml f32x2 [nsplit][bh*sq_tok] = {running max m_s, row sum l_s}, nsplit = ceil(sk_tok/keys_per_split);
 * qattn_int8_split_combine merges the splits into out f16 [rows, D] and lse f16 [rows] (rows =
 * bh*sq_tok): w_s = 2^(m_s - M) l_s, O = sum_s w_s opart_s / sum_s w_s, lse = f16(M + f16(log2 L)).
 * head_dim 128 only for the split forward (returns 1 otherwise). */
int qattn_int8_attn_fwd_split(const void* q_i8, const void* sq, const void* k_i8, const void* sk,
                              const void* vt, const void* sv, void* opart, void* ml, long bh,
                              long sq_tok, long sk_tok, int group, int keys_per_split, int head_dim,
                              float qks, void* stream);
int qattn_int8_split_combine(const void* opart, const void* ml, void* out, void* lse, long rows,
                             int nsplit, int head_dim, void* stream);

/* Backward prologue, one pass (attention_int8.py:372-374, 398): dO f16 -> dO_i8 [rows, D] + sdO f16
 * [rows/32] (same quantiser), dO_bf = bf16(dO_i8) [rows, D] (optional, NULL to skip), and LD f32x2
 * [rows] = {f32(lse), f32(f16(rowsum(dO*O)))}. */
int qattn_int8_bwd_prep(const void* dO, const void* O, const void* lse, void* dO_i8, void* sdO,
                        void* LD, void* dO_bf, long bh, long seq, int head_dim, void* stream);

/* Exact widening copy i8 -> bf16 of n elements (n % 16 == 0): the transposed-read operand images
 * of q_i8, k_i8, dO_i8 used by the dK / dQ / dV products (no reference counterpart). */
int qattn_i8_to_bf16(const void* x, void* y, long n, void* stream);

/* Corrected int8 backward (attention_int8.py:268-432 with SURVEY F4 fixed: dS = P*(dP - D),
 * sm_scale, deterministic per-head accumulation, k_mean term dropped since rowsum(dS) = 0).
 * Quantisation granularity as the reference: P and dS per 32x32 tile (amax/127, trunc), dO per
 * 32-row block, q/k/v int8 + scales from the forward.  Launches the dV, dK and dQ kernels.
 *   dq, dk, dv f16 [bh*seq, D] out; q_bf/k_bf/dO_bf = qattn_i8_to_bf16 images. */
int qattn_int8_attn_bwd(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                        const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                        const void* LD, const void* q_bf, const void* k_bf, const void* dO_bf,
                        void* dq, void* dk, void* dv, long bh, long seq, int head_dim, float qks,
                        float sms, void* stream);

/* qattn_int8_attn_bwd for the generalised shapes of qattn_int8_attn_fwd_ex: dq, dO and the
 * query-side tensors have bh heads of sq_tok rows, dk, dv and the key/value side bh / group heads of
 * sk_tok rows (dk, dv of a key/value head sum over its group of query heads). */
int qattn_int8_attn_bwd_ex(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                           const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                           const void* LD, const void* q_bf, const void* k_bf, const void* dO_bf,
                           void* dq, void* dk, void* dv, long bh, long sq_tok, long sk_tok, int group,
                           int causal, int head_dim, float qks, float sms, void* stream);

/* qattn_int8_attn_bwd_ex with a caller-provided dS workspace (no recomputation in the dQ pass):
 * the fused dK+dV kernel also stores each quantised 32x32 dS tile (dS_i8, 1 KiB, and its scale
 * s_dS) in ws, and the dQ kernel reads them back instead of recomputing S, dP, P and dS
 * (attention_int8.py:399-420).  dq, dk, dv are bit-identical to qattn_int8_attn_bwd_ex's.
 * ws must hold qattn_int8_bwd_ws_bytes(bh, sq_tok, sk_tok) bytes, 16-byte aligned; it is scratch
 * (overwritten, not read before written).  Returns 1 for ws == NULL. */
long qattn_int8_bwd_ws_bytes(long bh, long sq_tok, long sk_tok);
/* The largest dS-record workspace the backwards (int8 and bf16 alike) allocate before they fall back
 * to recomputation: QATTN_BWD_WS_MAX bytes if that is set, else 16 GiB (a workspace allocation
 * that fails also falls back to recomputation). */
long qattn_bwd_ws_cap(void);
int qattn_int8_attn_bwd_ws(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                           const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                           const void* LD, const void* q_bf, const void* k_bf, const void* dO_bf,
                           void* dq, void* dk, void* dv, void* ws, long bh, long sq_tok, long sk_tok,
                           int group, int causal, int head_dim, float qks, float sms, void* stream);

/* qattn_int8_attn_bwd_ws in chunks of kv_chunk key/value heads (each with its group query heads):
 * dK+dV then dQ per chunk, every chunk re-using the same ws, which must hold
 * qattn_int8_bwd_ws_bytes(kv_chunk * group, sq_tok, sk_tok) bytes.  Bit-identical to
 * qattn_int8_attn_bwd_ws; a chunk's records can stay in the Infinity Cache between the two passes.
 * Returns 1 for ws == NULL or kv_chunk < 1. */
int qattn_int8_attn_bwd_wsc(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                            const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                            const void* LD, const void* q_bf, const void* k_bf, const void* dO_bf,
                            void* dq, void* dk, void* dv, void* ws, long kv_chunk, long bh,
                            long sq_tok, long sk_tok, int group, int causal, int head_dim, float qks,
                            float sms, void* stream);

/* The two parts of qattn_int8_attn_bwd_ws (square, ungrouped, non-causal), launchable alone:
 * dK + dV writing the dS workspace, then dQ reading it. */
int qattn_int8_bwd_dkdv_ws(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                           const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                           const void* LD, const void* q_bf, const void* dO_bf, void* dk, void* dv,
                           void* ws, long bh, long seq, int head_dim, float qks, float sms,
                           void* stream);
int qattn_int8_bwd_dq_ws(const void* k_bf, const void* sk, void* dq, void* ws, long bh, long seq,
                         int head_dim, float sms, void* stream);

/* The parts of qattn_int8_attn_bwd, launchable alone (per-kernel timing / overlap):
 * dK and dV (attention_int8.py:375-378, 423-428), dV only, dK only, dQ only (414-420). */
int qattn_int8_bwd_dkdv(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                        const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                        const void* LD, const void* q_bf, const void* dO_bf, void* dk, void* dv,
                        long bh, long seq, int head_dim, float qks, float sms, void* stream);
int qattn_int8_bwd_dv(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                      const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                      const void* LD, const void* q_bf, const void* dO_bf, void* dk, void* dv,
                      long bh, long seq, int head_dim, float qks, float sms, void* stream);
int qattn_int8_bwd_dk(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                      const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                      const void* LD, const void* q_bf, const void* dO_bf, void* dk, void* dv,
                      long bh, long seq, int head_dim, float qks, float sms, void* stream);
int qattn_int8_bwd_dq(const void* dO_i8, const void* sdO, const void* q_i8, const void* sq,
                      const void* k_i8, const void* sk, const void* v_i8, const void* sv,
                      const void* LD, const void* k_bf, void* dq, long bh, long seq, int head_dim,
                      float qks, float sms, void* stream);

/* ---------------------------------------------------------------- bf16 path (attention_bf16.py) */

/* FA2 forward with the reference's "multiple-max" beta rule emulated per 16-key sub-tile
 * (helion_atten_bf16_fwd_training, attention_bf16.py:107-296).
 *   q, k f16 [bh*sq|sk, D]; v bf16 [bh*sk, D]; out O f32 [bh*sq, D]; lse f32 [bh*sq] (base 2).
 *   causal: strict-lower mask with fill -126 in raw logit units (attention_bf16.py:222-233).
 *   sq % 32 == 0, sk % 32 == 0. */
int qattn_bf16_fwd(const void* q, const void* k, const void* v, void* out, void* lse, long bh,
                   long sq, long sk, int head_dim, int causal, float qks, void* stream);

/* qattn_bf16_fwd with grouped-query attention: bh = batch * query heads, k and v
 * have bh / group heads (query head h reads key/value head h / group).  qattn_bf16_fwd is group = 1. */
int qattn_bf16_fwd_ex(const void* q, const void* k, const void* v, void* out, void* lse, long bh,
                      long sq, long sk, int group, int causal, int head_dim, float qks, void* stream);

/* Size in bytes of the V-suffix workspace of qattn_bf16_fwd_ws_ex: bh_kv*(sk/32+1)*head_dim*4. */
long qattn_bf16_fwd_ws_bytes(long bh_kv, long sk, int head_dim);
/* qattn_bf16_fwd_ex with a scratch workspace (16-byte aligned, qattn_bf16_fwd_ws_bytes(bh / group,
 * sk, head_dim) bytes) for the causal case: the per-head suffix sums of V are written there first and
 * replace the fully masked sub-tiles past each 32-query block's diagonal (whose P is one constant,
 * attention_bf16.py:222-285), so the causal forward streams half the key tiles.  Same outputs as
 * qattn_bf16_fwd_ex up to fp32 summation order.  Non-causal calls, and ws == NULL, ignore it. */
int qattn_bf16_fwd_ws_ex(const void* q, const void* k, const void* v, void* out, void* lse, long bh,
                         long sq, long sk, int group, int causal, int head_dim, float qks, void* ws,
                         void* stream);

/* Backward prologue, one pass: dO f32 -> dO_bf bf16 [rows, D] and LD f32x2 [rows] =
 * {lse[row], D = rowsum(dO*O)} (attention_bf16.py:416, computed once per row instead of per tile). */
int qattn_bf16_bwd_prep(const void* dO, const void* O, const void* lse, void* dO_bf, void* LD, long bh,
                        long seq, int head_dim, void* stream);

/* y = bf16(x) (round to nearest even) for n fp16 elements, n % 8 == 0: the transposed-read images of
 * q (dK product) and k (dQ product) of qattn_bf16_bwd (no reference counterpart). */
int qattn_f16_to_bf16(const void* x, void* y, long n, void* stream);

/* Corrected FA2 backward (helion_flash_atten_2_algo_4_bwd, attention_bf16.py:299-448 with SURVEY F3
 * fixed: dS = P*(dP - D), sm_scale, deterministic dq).  q, k f16; v bf16; dO_bf, LD from
 * qattn_bf16_bwd_prep; q_bf, k_bf = qattn_f16_to_bf16 images of q, k.  Out dq [bh*sq, D], dk, dv
 * [bh*sk, D] f32.  Launches one fused dK+dV kernel and one dQ kernel.  sq % 32 == 0,
 * sk % 32 == 0. */
int qattn_bf16_bwd(const void* q, const void* k, const void* v, const void* dO_bf, const void* LD,
                   const void* q_bf, const void* k_bf, void* dq, void* dk, void* dv, long bh, long sq,
                   long sk, int head_dim, int causal, float qks, float sms, void* stream);

/* qattn_bf16_bwd for grouped-query attention: dk, dv [bh/group * sk, D] sum over the group of
 * query heads of their key/value head; q_bf, k_bf as the query / key tensors. */
int qattn_bf16_bwd_ex(const void* q, const void* k, const void* v, const void* dO_bf, const void* LD,
                      const void* q_bf, const void* k_bf, void* dq, void* dk, void* dv, long bh, long sq,
                      long sk, int group, int causal, int head_dim, float qks, float sms, void* stream);

/* Size in bytes of the dS record workspace of qattn_bf16_bwd_ws_ex: bh*(sq/32)*(sk/32)*2048
 * (2 B per score), or -1 for sizes that are not multiples of 32. */
long qattn_bf16_bwd_ws_bytes(long bh, long sq, long sk);

/* qattn_bf16_bwd_ex whose fused dK+dV kernel also stores every bf16 dS tile in ws (device,
 * qattn_bf16_bwd_ws_bytes bytes) and whose dQ pass reads them instead of recomputing S and dP:
 * bit-identical dq, dk, dv. */
int qattn_bf16_bwd_ws_ex(const void* q, const void* k, const void* v, const void* dO_bf,
                         const void* LD, const void* q_bf, const void* k_bf, void* dq, void* dk,
                         void* dv, long bh, long sq, long sk, int group, int causal, int head_dim,
                         float qks, float sms, void* ws, void* stream);

/* qattn_bf16_bwd_ex with separate dV and dK kernels (each recomputes S; two waves per SIMD each):
 * bit-identical dk, dv to the fused kernel; kept for the parity test and as a timing reference. */
int qattn_bf16_bwd_split_ex(const void* q, const void* k, const void* v, const void* dO_bf,
                            const void* LD, const void* q_bf, const void* k_bf, void* dq, void* dk,
                            void* dv, long bh, long sq, long sk, int group, int causal, int head_dim,
                            float qks, float sms, void* stream);

/* ---------------------------------------------------------------- JVP (attention_jvp.py) */

/* Forward-mode tangent attention (helion_attention_jvp_forward_fp32, attention_jvp.py:24-195):
 *   q, k, v, tq, tk, tv bf16 [bh*sq|sk, D]; out O, tO f32 [bh*sq, D]; lse f32 [bh*sq] (base 2).
 *   tO = (P.tV + (P o tS).V - rowsum(P o tS) * O) / l with tS = (tq.k^T + q.tk^T) * sm.
 *   flags must be 0 (reserved).  sq % 32 == 0, sk % 64 == 0. */
int qattn_jvp_fwd(const void* q, const void* k, const void* v, const void* tq, const void* tk,
                  const void* tv, void* out, void* tout, void* lse, long bh, long sq, long sk,
                  int head_dim, int flags, float qks, float sm, void* stream);

/* fp32-accurate JVP (the reference's fp32 contract, SURVEY §8c "fp32 mode"): every operand is given
 * as two bf16 images x = hi + lo (qattn_split_bf16) and every product runs as
 * hi*hi + hi*lo + lo*hi + lo*lo on the bf16 MFMA (exact up to the 2^-17 split residual, fp32
 * accumulation).  Same outputs and
 * conventions as qattn_jvp_fwd; sq % 32 == 0, sk % 32 == 0. */
int qattn_jvp_fwd_x3(const void* q_hi, const void* q_lo, const void* k_hi, const void* k_lo,
                     const void* v_hi, const void* v_lo, const void* tq_hi, const void* tq_lo,
                     const void* tk_hi, const void* tk_lo, const void* tv_hi, const void* tv_lo,
                     void* out, void* tout, void* lse, long bh, long sq, long sk, int head_dim,
                     float qks, float sm, void* stream);

/* qattn_jvp_fwd / qattn_jvp_fwd_x3 with grouped-query attention (SURVEY §8f N2 for the JVP path):
 * bh = batch * query heads; k, v, tk, tv have bh / group heads (query head h reads key/value head
 * h / group).  The reference's JVP kernel takes equal head counts (jvp:33-41). */
int qattn_jvp_fwd_ex(const void* q, const void* k, const void* v, const void* tq, const void* tk,
                     const void* tv, void* out, void* tout, void* lse, long bh, long sq, long sk,
                     int group, int head_dim, float qks, float sm, void* stream);
int qattn_jvp_fwd_x3_ex(const void* q_hi, const void* q_lo, const void* k_hi, const void* k_lo,
                        const void* v_hi, const void* v_lo, const void* tq_hi, const void* tq_lo,
                        const void* tk_hi, const void* tk_lo, const void* tv_hi, const void* tv_lo,
                        void* out, void* tout, void* lse, long bh, long sq, long sk, int group,
                        int head_dim, float qks, float sm, void* stream);

/* Primal-only forward of the JVP kernel (O, lse; no tangent operands or chains): the forward of
 * AttentionJVP_autograd_function, whose jvp() then runs qattn_jvp_fwd_ex once.
 * O / lse are bit-identical to those qattn_jvp_fwd_ex / qattn_jvp_fwd_x3_ex return for the same
 * primals.  Arguments as those entries without the tangents. */
int qattn_jvp_primal_ex(const void* q, const void* k, const void* v, void* out, void* lse, long bh,
                        long sq, long sk, int group, int head_dim, float qks, float sm, void* stream);
int qattn_jvp_primal_x3_ex(const void* q_hi, const void* q_lo, const void* k_hi, const void* k_lo,
                           const void* v_hi, const void* v_lo, void* out, void* lse, long bh, long sq,
                           long sk, int group, int head_dim, float qks, float sm, void* stream);

/* hi = bf16(x), lo = bf16(x - hi) (both round-to-nearest-even) for n fp32 elements, n % 4 == 0. */
int qattn_split_bf16(const void* x, void* hi, void* lo, long n, void* stream);

/* ---------------------------------------------------------------- MX-FP4 inference forward
 * SURVEY §8f N4 (SageAttention3's FP4 path, named in the reference README.md:49-55, not implemented
 * there: no reference interface is replaced).  OCP MX e2m1 with one e8m0 scale per 32 elements,
 * e = floor(log2 amax) - 2, code = RNE(sat(x / 2^e)); layouts in csrc/mxfp4_attn.hip. */

/* Q / K rows: x f16 [rows, head_dim] -> q4 u8 [rows, head_dim/2] (low nibble first), scale u8
 * [rows, head_dim/32].  mean (f16 [rows/seq, head_dim]) or NULL: when given, row r is first
 * smoothed to f16(x - mean[r / seq]) (k_mean from qattn_kmean).  head_dim 64 or 128. */
int qattn_mxfp4_quant_rows(const void* x, const void* mean, void* q4, void* scale, long rows, long seq,
                           int head_dim, void* stream);

/* V: v f16 [bh*seq, head_dim] -> vt u8 [bh][seq/64][head_dim][32] (operand-ordered keys), vscale u8
 * [bh][seq/64][head_dim][2].  seq % 64 == 0. */
int qattn_mxfp4_quant_vt(const void* v, void* vt, void* vscale, long bh, long seq, int head_dim,
                         void* stream);

/* O f16 [bh*sq, 128] = softmax2(S * qks) V with S from the fp4 Q/K, P re-quantised to fp4 per
 * 32 keys, l from the fp32 P; lse f32 [bh*sq] (base 2).  Query head h reads key/value head h/group.
 * sq % 32 == 0, sk % 64 == 0, head_dim 128. */
int qattn_mxfp4_attn_fwd(const void* q4, const void* qscale, const void* k4, const void* kscale,
                         const void* vt, const void* vscale, void* out, void* lse, long bh, long sq,
                         long sk, int group, int head_dim, float qks, void* stream);

/* Fragment-layout probes and other diagnostics live in a separate development library
 * (libqattn_dev.so, include/qattn_dev.h); this library exports the product API only. */

#ifdef __cplusplus
}
#endif

#endif /* QATTN_H */
