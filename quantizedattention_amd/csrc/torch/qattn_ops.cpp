// TORCH_LIBRARY(qattn) operator layer over the C-ABI kernel library ("C++ op layer").
//
// Each operator allocates its outputs on the inputs' device, enters a HIP device guard on that
// device (c10::hip::HIPGuardMasqueradingAsCUDA: ROCm torch reports HIP devices as 'cuda') and
// enqueues the kernels of include/qattn.h on torch's current stream of that device
// (c10::hip::getCurrentHIPStream, c10/hip/HIPStream.h:245).  The kernel sequences are those of the
// Python drop-in functions (attention_int8.py / attention_bf16.py / attention_jvp.py /
// attention_mxfp4.py), so an operator's outputs are bit-identical to the drop-in's
// (tests/test_gpu_ops.py).  Registered for the CUDA dispatch key only: there is no CPU kernel, as
// in the drop-ins; the Python side (quantizedattention_amd/ops.py) adds the fake (meta)
// implementations and the autograd rules of int8_fwd / bf16_fwd.
//
// Schemas (reference file:line of the computation each replaces):
//   int8_quant(Tensor x, int block) -> (Tensor, Tensor)                 attention_int8.py:178-186
//   int8_fwd(Tensor q, Tensor k, Tensor v, bool smooth, bool causal)   attention_int8.py:20-65, 97-262
//       -> (O, lse, q_i8, k_i8, v_i8, sq, sk, sv)        (k_i8 row-major [B*Hkv*Sk, D])
//   int8_bwd(dO, q_i8, sq, k_i8, sk, v_i8, sv, O, lse, bool causal, int kv_heads)
//       -> (dq, dk, dv)                                                  attention_int8.py:264-432
//   bf16_fwd(q, k, v, bool causal) -> (O, lse)                           attention_bf16.py:107-296
//   bf16_bwd(q, k, v, O, lse, bool causal, dO) -> (dq, dk, dv)           attention_bf16.py:299-448
//   jvp_fwd(q, k, v, tq, tk, tv) -> (O, tO, lse)                         attention_jvp.py:24-195
//   mxfp4_fwd(q, k, v) -> O                                  (README.md:49-55)
// Errors: TORCH_CHECK (c10::Error, RuntimeError in Python) with the drop-ins' messages; int8_quant's
// argument checks raise ValueError (TORCH_CHECK_VALUE) as its Python predecessor did.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <c10/hip/HIPCachingAllocator.h>

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>

#include "qattn.h"

namespace {

using at::Tensor;
using T3 = std::tuple<Tensor, Tensor, Tensor>;

void* P(const Tensor& t) { return t.defined() ? t.data_ptr() : nullptr; }

struct Ctx {   // device guard + the current stream of the inputs' device
  c10::hip::HIPGuardMasqueradingAsCUDA guard;
  void* stream;
  explicit Ctx(const Tensor& t)
      : guard(t.device()), stream((void*)c10::hip::getCurrentHIPStream(t.device().index()).stream()) {}
};

void call(int rc, const char* what) {
  TORCH_CHECK(rc != 1, "qattn: ", what, ": unsupported shape");
  TORCH_CHECK(rc == 0, "qattn: ", what, ": kernel launch failed");
}

void require_gpu(std::initializer_list<const Tensor*> ts) {
  for (const Tensor* t : ts)
    TORCH_CHECK(t->is_cuda(), "qattn kernels run on the GPU only; got a tensor on ", t->device(),
                " (no CPU fallback by design)");
}

// fp32(1/sqrt(D) * log2(e)) and fp32(1/sqrt(D)): the Python double rounded once to fp32
float qk_scale(int64_t D) { return (float)(1.0 / std::sqrt((double)D) * 1.44269504); }
float sm_scale(int64_t D) { return (float)(1.0 / std::sqrt((double)D)); }

int64_t env_i64(const char* name, int64_t dflt) {
  const char* s = std::getenv(name);
  return (s && *s) ? std::strtoll(s, nullptr, 10) : dflt;
}

Tensor empty(at::IntArrayRef shape, at::ScalarType dt, const Tensor& like) {
  return at::empty(shape, like.options().dtype(dt));
}

// A backward workspace of `bytes`, undefined when the allocator refuses.  torch's caching allocator
// frees every cached block and retries before it raises, so after one refusal a workspace that large
// is tried again only when the device has room for it (hipMemGetInfo free bytes plus the allocator's
// reserved-but-unused bytes): a training loop whose workspace never fits does not flush the cache in
// every backward (the same rule as _lib.try_workspace).
Tensor try_empty(int64_t bytes, const Tensor& like) {
  static std::mutex mu;
  static std::map<int, int64_t> refused;   // device -> smallest refused size
  const int dev = like.device().index();
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = refused.find(dev);
    if (it != refused.end() && bytes >= it->second) {
      size_t free_b = 0, total_b = 0;
      const auto st = c10::hip::HIPCachingAllocator::getDeviceStats(dev);
      const int64_t spare = st.reserved_bytes[0].current - st.allocated_bytes[0].current;
      if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || (int64_t)free_b + spare < bytes)
        return Tensor();
    }
  }
  try {
    Tensor t = at::empty({bytes}, like.options().dtype(at::kByte));
    std::lock_guard<std::mutex> g(mu);
    auto it = refused.find(dev);
    if (it != refused.end() && bytes >= it->second) refused.erase(it);
    return t;
  } catch (const c10::OutOfMemoryError&) {
    std::lock_guard<std::mutex> g(mu);
    auto it = refused.find(dev);
    if (it == refused.end() || bytes < it->second) refused[dev] = bytes;
    return Tensor();
  }
}

// ------------------------------------------------------------------------------------ int8
std::tuple<Tensor, Tensor> int8_quant(const Tensor& x, int64_t block) {
  TORCH_CHECK_VALUE(block == 32, "qattn::int8_quant supports block = 32 (the reference's Bq = Bkv)");
  TORCH_CHECK_VALUE(x.dim() >= 2 && x.size(-2) % 32 == 0 && (x.size(-1) == 64 || x.size(-1) == 128),
              "qattn::int8_quant needs x [..., S, D] with S % 32 == 0 and D in (64, 128)");
  require_gpu({&x});
  Ctx c(x);
  const Tensor xh = x.to(at::kHalf).contiguous();
  const int64_t D = x.size(-1), rows = xh.numel() / D, S = x.size(-2);
  Tensor idx = empty(xh.sizes(), at::kChar, xh);
  std::vector<int64_t> ss(xh.sizes().begin(), xh.sizes().end() - 2);
  ss.push_back(S / 32);
  Tensor scale = empty(ss, at::kHalf, xh);
  if (rows == 0) return {idx, scale};
  call(qattn_int8_quant(P(xh), P(idx), P(scale), nullptr, nullptr, rows, (int)S, (int)D, c.stream),
       "int8_quant");
  return {idx, scale};
}

void check_int8(const Tensor& q, const Tensor& k, const Tensor& v) {
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "qattn int8: q, k, v must be [B, H, S, D]");
  TORCH_CHECK(k.size(2) == v.size(2), "k and v tokens are different");          // int8:126
  TORCH_CHECK(k.size(3) == v.size(3), "k head_dim and v head_dim are different");  // int8:127
  TORCH_CHECK(q.size(0) == k.size(0) && k.sizes().slice(0, 2) == v.sizes().slice(0, 2) &&
                  q.size(3) == k.size(3) && q.size(1) % k.size(1) == 0,
              "qattn int8: batch and head_dim must match and q heads must be a multiple of k/v heads");
  TORCH_CHECK(q.size(2) % 32 == 0 && k.size(2) % 32 == 0, "qattn int8: token counts must be multiples of 32");
  TORCH_CHECK(q.size(3) == 64 || q.size(3) == 128, "qattn int8: head_dim must be 64 or 128");
}

using T8 = std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor>;

// attention_int8._int8_forward
T8 int8_fwd(const Tensor& q_in, const Tensor& k_in, const Tensor& v_in, bool smooth, bool causal) {
  check_int8(q_in, k_in, v_in);
  require_gpu({&q_in, &k_in, &v_in});
  Ctx c(q_in);
  const Tensor q = q_in.to(at::kHalf).contiguous(), k = k_in.to(at::kHalf).contiguous(),
               v = v_in.to(at::kHalf).contiguous();
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  const int64_t Hkv = k.size(1), Sk = k.size(2), N = B * H * S, Nkv = B * Hkv * Sk;
  Tensor q_i8 = empty({N, D}, at::kChar, q), k_i8 = empty({Nkv, D}, at::kChar, q),
         v_i8 = empty({Nkv, D}, at::kChar, q);
  Tensor sq = empty({N / 32}, at::kHalf, q), sk = empty({Nkv / 32}, at::kHalf, q),
         sv = empty({Nkv / 32}, at::kHalf, q);
  Tensor vt = empty({Nkv, D}, at::kChar, q);   // the int8 V^T operand image
  Tensor O = empty({B, H, S, D}, at::kHalf, q), lse = empty({N}, at::kHalf, q);
  Tensor k_mean;
  if (N == 0 || Nkv == 0) {   // an empty problem: nothing to read, zero outputs
    O.zero_();
    lse.zero_();
    return {O, lse, q_i8, k_i8, v_i8, sq, sk, sv};
  }
  if (smooth) {
    k_mean = empty({B, Hkv, 1, D}, at::kHalf, q);
    call(qattn_kmean(P(k), P(k_mean), B * Hkv, Sk, (int)D, c.stream), "kmean");
  }

  const float qks = qk_scale(D);
  call(qattn_int8_quant(P(k), P(k_i8), P(sk), nullptr, P(k_mean), Nkv, (int)Sk, (int)D, c.stream),
       "quantise k");
  call(qattn_int8_quant_vt(P(v), P(v_i8), P(sv), P(vt), Nkv, (int)D, c.stream), "quantise v");
  call(qattn_int8_attn_fwd_qf(P(q), P(q_i8), P(sq), nullptr, P(k_i8), P(sk), P(vt), P(sv), P(O), P(lse),
                              B * H, S, Sk, (int)(H / Hkv), causal ? 1 : 0, (int)D, qks, c.stream),
       "int8 forward");
  return {O, lse, q_i8, k_i8, v_i8, sq, sk, sv};
}

// attention_int8._int8_backward: dS-record workspace (in head chunks when not causal) by default,
// recomputation when the workspace does not fit
T3 int8_bwd(const Tensor& dO_in, const Tensor& q_i8_in, const Tensor& sq, const Tensor& k_i8_in,
            const Tensor& sk, const Tensor& v_i8_in, const Tensor& sv, const Tensor& O_in,
            const Tensor& lse_in, bool causal, int64_t kv_heads) {
  require_gpu({&dO_in, &q_i8_in, &O_in});
  TORCH_CHECK(O_in.dim() == 4, "qattn int8 backward: O must be [B, H, S, D]");
  Ctx c(O_in);
  const Tensor O = O_in.to(at::kHalf).contiguous(), dO = dO_in.to(at::kHalf).contiguous();
  const int64_t B = O.size(0), H = O.size(1), S = O.size(2), D = O.size(3), Hkv = kv_heads;
  const int64_t Nkv = k_i8_in.size(0);
  if (B * H * S == 0 || Nkv == 0) {   // nothing attends: zero gradients
    TORCH_CHECK(Hkv > 0, "qattn int8 backward: inconsistent key/value heads");
    const int64_t Sk0 = B * Hkv ? Nkv / (B * Hkv) : 0;
    auto z = O_in.options().dtype(at::kHalf);
    return {at::zeros({B, H, S, D}, z), at::zeros({B, Hkv, Sk0, D}, z), at::zeros({B, Hkv, Sk0, D}, z)};
  }
  TORCH_CHECK(Hkv > 0 && H % Hkv == 0 && Nkv % (B * Hkv) == 0,
              "qattn int8 backward: inconsistent key/value heads");
  const int64_t Sk = Nkv / (B * Hkv), N = B * H * S, G = H / Hkv;
  const Tensor q_i8 = q_i8_in.contiguous(), k_i8 = k_i8_in.contiguous(), v_i8 = v_i8_in.contiguous();
  const Tensor sqc = sq.contiguous(), skc = sk.contiguous(), svc = sv.contiguous();
  const Tensor lse = lse_in.to(at::kHalf).contiguous();
  Tensor dO_i8 = empty({N, D}, at::kChar, O), sdO = empty({N / 32}, at::kHalf, O);
  Tensor LD = empty({N, 2}, at::kFloat, O), dO_bf = empty({N, D}, at::kBFloat16, O);
  call(qattn_int8_bwd_prep(P(dO), P(O), P(lse), P(dO_i8), P(sdO), P(LD), P(dO_bf), B * H, S, (int)D,
                           c.stream),
       "int8 backward prep");
  Tensor q_bf = empty({N, D}, at::kBFloat16, O), k_bf = empty({Nkv, D}, at::kBFloat16, O);
  call(qattn_i8_to_bf16(P(q_i8), P(q_bf), N * D, c.stream), "q image");
  call(qattn_i8_to_bf16(P(k_i8), P(k_bf), Nkv * D, c.stream), "k image");
  Tensor dq = empty({B, H, S, D}, at::kHalf, O), dk = empty({B, Hkv, Sk, D}, at::kHalf, O),
         dv = empty({B, Hkv, Sk, D}, at::kHalf, O);
  const float qks = qk_scale(D), sms = sm_scale(D);
  // workspace chunking (attention_int8._ws_chunk): non-causal >= 512 dK+dV workgroups per chunk
  const int64_t bkv = B * Hkv;
  int64_t chunk = env_i64("QATTN_BWD_WS_CHUNK", -1);
  if (chunk < 0) chunk = causal ? 0 : (512 + std::max<int64_t>(1, Sk / 256) - 1) / std::max<int64_t>(1, Sk / 256);
  chunk = chunk <= 0 ? bkv : std::min(chunk, bkv);
  const int64_t ws_bytes = qattn_int8_bwd_ws_bytes(chunk * G, S, Sk);
  const bool region_ok = G * (S / 32) * (Sk / 32) * 1024 < (int64_t(1) << 31);
  Tensor ws;
  if (ws_bytes > 0 && region_ok && ws_bytes <= qattn_bwd_ws_cap())
    ws = try_empty(ws_bytes, O);
  if (ws.defined() && chunk < bkv) {
    call(qattn_int8_attn_bwd_wsc(P(dO_i8), P(sdO), P(q_i8), P(sqc), P(k_i8), P(skc), P(v_i8), P(svc),
                                 P(LD), P(q_bf), P(k_bf), P(dO_bf), P(dq), P(dk), P(dv), P(ws), chunk,
                                 B * H, S, Sk, (int)G, causal ? 1 : 0, (int)D, qks, sms, c.stream),
         "int8 backward");
  } else if (ws.defined()) {
    call(qattn_int8_attn_bwd_ws(P(dO_i8), P(sdO), P(q_i8), P(sqc), P(k_i8), P(skc), P(v_i8), P(svc),
                                P(LD), P(q_bf), P(k_bf), P(dO_bf), P(dq), P(dk), P(dv), P(ws), B * H, S,
                                Sk, (int)G, causal ? 1 : 0, (int)D, qks, sms, c.stream),
         "int8 backward");
  } else {
    call(qattn_int8_attn_bwd_ex(P(dO_i8), P(sdO), P(q_i8), P(sqc), P(k_i8), P(skc), P(v_i8), P(svc),
                                P(LD), P(q_bf), P(k_bf), P(dO_bf), P(dq), P(dk), P(dv), B * H, S, Sk,
                                (int)G, causal ? 1 : 0, (int)D, qks, sms, c.stream),
         "int8 backward");
  }
  return {dq, dk, dv};
}

// ------------------------------------------------------------------------------------ bf16
void check_bf16(const Tensor& q, const Tensor& k, const Tensor& v) {
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "qattn bf16: q, k, v must be [B, H, S, D]");
  TORCH_CHECK(k.size(2) == v.size(2), "input k_tokens must match v_tokens");   // bf16:154
  TORCH_CHECK(q.size(3) == k.size(3) && k.size(3) == v.size(3),
              "all head dimensions must match for q, k, v tensors");          // bf16:155
  TORCH_CHECK(q.size(0) == k.size(0) && k.sizes().slice(0, 2) == v.sizes().slice(0, 2) &&
                  q.size(1) % k.size(1) == 0,
              "qattn bf16: batch must match and q heads must be a multiple of k/v heads");
  TORCH_CHECK(q.size(2) % 32 == 0 && k.size(2) % 32 == 0, "qattn bf16: token counts must be multiples of 32");
  TORCH_CHECK(q.size(3) == 64 || q.size(3) == 128, "qattn bf16: head_dim must be 64 or 128");
}

std::tuple<Tensor, Tensor> bf16_fwd(const Tensor& q_in, const Tensor& k_in, const Tensor& v_in,
                                    bool causal) {
  check_bf16(q_in, k_in, v_in);
  require_gpu({&q_in, &k_in, &v_in});
  Ctx c(q_in);
  const Tensor q = q_in.to(at::kHalf).contiguous(), k = k_in.to(at::kHalf).contiguous(),
               v = v_in.to(at::kBFloat16).contiguous();
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3), Sk = k.size(2);
  Tensor O = empty({B, H, S, D}, at::kFloat, q), lse = empty({B * H, S}, at::kFloat, q);
  if (O.numel() == 0 || k.numel() == 0) return {O.zero_(), lse.zero_()};
  // causal: the per-head V suffix sums stand in for the fully masked key tiles (include/qattn.h);
  // without room for them the kernel runs the whole masked tile loop (same results)
  Tensor ws;
  if (causal) ws = try_empty(qattn_bf16_fwd_ws_bytes(B * k.size(1), Sk, (int)D), q);
  call(qattn_bf16_fwd_ws_ex(P(q), P(k), P(v), P(O), P(lse), B * H, S, Sk, (int)(H / k.size(1)),
                            causal ? 1 : 0, (int)D, qk_scale(D), P(ws), c.stream),
       "bf16 forward");
  return {O, lse};
}

// attention_bf16.helion_flash_atten_2_algo_4_bwd (entry "auto": causal -> dS records)
T3 bf16_bwd(const Tensor& q_in, const Tensor& k_in, const Tensor& v_in, const Tensor& O_in,
            const Tensor& lse_in, bool causal, const Tensor& dO_in) {
  check_bf16(q_in, k_in, v_in);
  require_gpu({&q_in, &k_in, &v_in, &O_in, &lse_in, &dO_in});
  Ctx c(q_in);
  const Tensor q = q_in.to(at::kHalf).contiguous(), k = k_in.to(at::kHalf).contiguous(),
               v = v_in.to(at::kBFloat16).contiguous(), O = O_in.to(at::kFloat).contiguous(),
               dO = dO_in.to(at::kFloat).contiguous(), lse = lse_in.to(at::kFloat).contiguous();
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3);
  const int64_t Hkv = k.size(1), Sk = k.size(2);
  if (q.numel() == 0 || k.numel() == 0) {   // nothing attends: zero gradients
    auto z = q.options().dtype(at::kFloat);
    return {at::zeros(q.sizes(), z), at::zeros(k.sizes(), z), at::zeros(v.sizes(), z)};
  }
  Tensor dO_bf = empty({B, H, S, D}, at::kBFloat16, q), LD = empty({B * H, S, 2}, at::kFloat, q);
  call(qattn_bf16_bwd_prep(P(dO), P(O), P(lse), P(dO_bf), P(LD), B * H, S, (int)D, c.stream),
       "bf16 backward prep");
  Tensor q_bf = empty(q.sizes(), at::kBFloat16, q), k_bf = empty(k.sizes(), at::kBFloat16, q);
  call(qattn_f16_to_bf16(P(q), P(q_bf), q.numel(), c.stream), "q image");
  call(qattn_f16_to_bf16(P(k), P(k_bf), k.numel(), c.stream), "k image");
  Tensor dq = empty({B, H, S, D}, at::kFloat, q), dk = empty({B, Hkv, Sk, D}, at::kFloat, q),
         dv = empty({B, Hkv, Sk, D}, at::kFloat, q);
  const float qks = qk_scale(D), sms = sm_scale(D);
  const int64_t forced = env_i64("QATTN_BF16_BWD_WS", -1);   // 1 / 0 force the records on / off
  const bool want_ws = forced < 0 ? causal : forced == 1;
  Tensor ws;
  if (want_ws) {
    const int64_t ws_bytes = qattn_bf16_bwd_ws_bytes(B * H, S, Sk);
    if (ws_bytes > 0 && ws_bytes <= qattn_bwd_ws_cap()) ws = try_empty(ws_bytes, q);
  }
  if (ws.defined())
    call(qattn_bf16_bwd_ws_ex(P(q), P(k), P(v), P(dO_bf), P(LD), P(q_bf), P(k_bf), P(dq), P(dk), P(dv),
                              B * H, S, Sk, (int)(H / Hkv), causal ? 1 : 0, (int)D, qks, sms, P(ws),
                              c.stream),
         "bf16 backward");
  else
    call(qattn_bf16_bwd_ex(P(q), P(k), P(v), P(dO_bf), P(LD), P(q_bf), P(k_bf), P(dq), P(dk), P(dv),
                           B * H, S, Sk, (int)(H / Hkv), causal ? 1 : 0, (int)D, qks, sms, c.stream),
         "bf16 backward");
  return {dq, dk, dv};
}

// ------------------------------------------------------------------------------------- jvp
// attention_jvp._jvp: bf16 inputs on the bf16 MFMA, other dtypes as fp32 split into bf16 hi/lo
T3 jvp_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& tq, const Tensor& tk,
           const Tensor& tv) {
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "qattn jvp: q, k, v must be [B, H, S, D]");
  TORCH_CHECK(k.size(2) == v.size(2), "input k_tokens must match v_tokens");   // jvp:78
  TORCH_CHECK(q.size(3) == k.size(3) && k.size(3) == v.size(3),
              "all head dimensions must match for q, k, v tensors");          // jvp:79
  require_gpu({&q, &k, &v, &tq, &tk, &tv});
  TORCH_CHECK(q.size(2) % 32 == 0 && k.size(2) % 32 == 0, "qattn jvp: q and k tokens must be multiples of 32");
  TORCH_CHECK(q.size(3) == 64 || q.size(3) == 128, "qattn jvp: head_dim must be 64 or 128");
  TORCH_CHECK(tq.sizes() == q.sizes() && tk.sizes() == k.sizes() && tv.sizes() == v.sizes(),
              "qattn jvp: tangents must have the primals' shapes");
  const int64_t B = q.size(0), H = q.size(1), S = q.size(2), D = q.size(3), Hkv = k.size(1);
  const int64_t Sk = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Hkv && H % Hkv == 0,
              "qattn jvp: k and v need q's batch and a head count dividing q's");
  Ctx c(q);
  Tensor O = empty({B, H, S, D}, at::kFloat, q), tO = empty({B, H, S, D}, at::kFloat, q),
         lse = empty({B * H, S}, at::kFloat, q);
  if (O.numel() == 0 || k.numel() == 0) return {O.zero_(), tO.zero_(), lse.zero_()};
  const float qks = qk_scale(D), sm = sm_scale(D);
  const int G = (int)(H / Hkv);
  const Tensor* ins[6] = {&q, &k, &v, &tq, &tk, &tv};
  bool all_bf16 = true;
  for (const Tensor* t : ins) all_bf16 = all_bf16 && t->scalar_type() == at::kBFloat16;
  if (all_bf16) {
    TORCH_CHECK(Sk % 64 == 0, "qattn jvp: k tokens must be a multiple of 64 for bf16 inputs");
    Tensor x[6];
    for (int i = 0; i < 6; ++i) x[i] = ins[i]->contiguous();
    call(qattn_jvp_fwd_ex(P(x[0]), P(x[1]), P(x[2]), P(x[3]), P(x[4]), P(x[5]), P(O), P(tO), P(lse), B * H,
                          S, Sk, G, (int)D, qks, sm, c.stream),
         "jvp forward");
    return {O, tO, lse};
  }
  Tensor hi[6], lo[6];
  for (int i = 0; i < 6; ++i) {
    const Tensor x = ins[i]->to(at::kFloat).contiguous();
    hi[i] = empty(x.sizes(), at::kBFloat16, x);
    lo[i] = empty(x.sizes(), at::kBFloat16, x);
    call(qattn_split_bf16(P(x), P(hi[i]), P(lo[i]), x.numel(), c.stream), "split fp32");
  }
  call(qattn_jvp_fwd_x3_ex(P(hi[0]), P(lo[0]), P(hi[1]), P(lo[1]), P(hi[2]), P(lo[2]), P(hi[3]), P(lo[3]),
                           P(hi[4]), P(lo[4]), P(hi[5]), P(lo[5]), P(O), P(tO), P(lse), B * H, S, Sk, G,
                           (int)D, qks, sm, c.stream),
       "jvp forward");
  return {O, tO, lse};
}

// ----------------------------------------------------------------------------------- mxfp4
// attention_mxfp4.mxfp4_attn_fwd with k smoothing (sage_attention_3_fp4)
Tensor mxfp4_fwd(const Tensor& q_in, const Tensor& k_in, const Tensor& v_in) {
  TORCH_CHECK(q_in.dim() == 4 && k_in.sizes() == v_in.sizes() && q_in.size(0) == k_in.size(0) &&
                  q_in.size(-1) == k_in.size(-1),
              "qattn mxfp4: q [B,H,Sq,D], k = v [B,Hkv,Sk,D] expected");
  TORCH_CHECK(q_in.size(1) % k_in.size(1) == 0, "qattn mxfp4: query heads must be a multiple of key/value heads");
  TORCH_CHECK(q_in.size(-1) == 128, "qattn mxfp4: head_dim must be 128");
  TORCH_CHECK(q_in.size(2) % 32 == 0 && k_in.size(2) % 64 == 0,
              "qattn mxfp4: q tokens must be a multiple of 32, k tokens of 64");
  require_gpu({&q_in, &k_in, &v_in});
  Ctx c(q_in);
  const Tensor q = q_in.to(at::kHalf).contiguous(), k = k_in.to(at::kHalf).contiguous(),
               v = v_in.to(at::kHalf).contiguous();
  const int64_t B = q.size(0), H = q.size(1), Sq = q.size(2), D = q.size(3), Hkv = k.size(1),
                Sk = k.size(2);
  if (q.numel() == 0 || k.numel() == 0) return at::zeros({B, H, Sq, D}, q.options());
  Tensor k_mean = empty({B, Hkv, 1, D}, at::kHalf, q);
  call(qattn_kmean(P(k), P(k_mean), B * Hkv, Sk, (int)D, c.stream), "kmean");
  Tensor q4 = empty({B * H * Sq, D / 2}, at::kByte, q), qs = empty({B * H * Sq, D / 32}, at::kByte, q);
  Tensor k4 = empty({B * Hkv * Sk, D / 2}, at::kByte, q), ks = empty({B * Hkv * Sk, D / 32}, at::kByte, q);
  call(qattn_mxfp4_quant_rows(P(q), nullptr, P(q4), P(qs), B * H * Sq, Sq, (int)D, c.stream), "quantise q");
  call(qattn_mxfp4_quant_rows(P(k), P(k_mean), P(k4), P(ks), B * Hkv * Sk, Sk, (int)D, c.stream),
       "quantise k");
  Tensor vt = empty({B * Hkv, Sk / 64, D, 32}, at::kByte, q), vs = empty({B * Hkv, Sk / 64, D, 2}, at::kByte, q);
  call(qattn_mxfp4_quant_vt(P(v), P(vt), P(vs), B * Hkv, Sk, (int)D, c.stream), "quantise v");
  Tensor out = empty({B, H, Sq, D}, at::kHalf, q), lse = empty({B * H, Sq}, at::kFloat, q);
  call(qattn_mxfp4_attn_fwd(P(q4), P(qs), P(k4), P(ks), P(vt), P(vs), P(out), P(lse), B * H, Sq, Sk,
                            (int)(H / Hkv), (int)D, qk_scale(D), c.stream),
       "mxfp4 forward");
  return out;
}

}  // namespace

TORCH_LIBRARY(qattn, m) {
  m.def("int8_quant(Tensor x, int block) -> (Tensor, Tensor)");
  m.def("int8_fwd(Tensor q, Tensor k, Tensor v, bool smooth, bool causal) -> "
        "(Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("int8_bwd(Tensor dO, Tensor q_i8, Tensor sq, Tensor k_i8, Tensor sk, Tensor v_i8, Tensor sv, "
        "Tensor O, Tensor lse, bool causal, int kv_heads) -> (Tensor, Tensor, Tensor)");
  m.def("bf16_fwd(Tensor q, Tensor k, Tensor v, bool causal) -> (Tensor, Tensor)");
  m.def("bf16_bwd(Tensor q, Tensor k, Tensor v, Tensor O, Tensor lse, bool causal, Tensor dO) -> "
        "(Tensor, Tensor, Tensor)");
  m.def("jvp_fwd(Tensor q, Tensor k, Tensor v, Tensor tq, Tensor tk, Tensor tv) -> (Tensor, Tensor, Tensor)");
  m.def("mxfp4_fwd(Tensor q, Tensor k, Tensor v) -> Tensor");
}

TORCH_LIBRARY_IMPL(qattn, CUDA, m) {
  m.impl("int8_quant", &int8_quant);
  m.impl("int8_fwd", &int8_fwd);
  m.impl("int8_bwd", &int8_bwd);
  m.impl("bf16_fwd", &bf16_fwd);
  m.impl("bf16_bwd", &bf16_bwd);
  m.impl("jvp_fwd", &jvp_fwd);
  m.impl("mxfp4_fwd", &mxfp4_fwd);
}
