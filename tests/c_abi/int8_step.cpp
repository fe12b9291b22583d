// A non-Python host of the C ABI (include/qattn.h): the int8 SageAttention-3 training step of
// INTEGRATION.md §3 -- k-smoothing, quantisers (with the backward's bf16 images), the int8 forward
// with P.V on the int8 MFMA, the backward prologue and the dS-record backward -- on raw f16 files,
// with no torch anywhere.  tests/test_gpu_c_abi.py runs it and compares every output bit for bit with
// the Python drop-in (sage_attention_3_int8's forward + backward path).
//
//   int8_step <B> <H> <S> <D> <dir>    reads  dir/{q,k,v,dO}.f16  ([B,H,S,D] row-major fp16)
//                                      writes dir/{O,lse,dq,dk,dv}.f16
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "qattn.h"

#define CHECK_HIP(x)                                                           \
  do {                                                                         \
    if ((x) != hipSuccess) { std::fprintf(stderr, "HIP error at %d\n", __LINE__); std::exit(3); } \
  } while (0)
#define CHECK_QA(x)                                                                    \
  do {                                                                                 \
    const int rc_ = (x);                                                               \
    if (rc_ != 0) { std::fprintf(stderr, "qattn call failed (%d) at %d\n", rc_, __LINE__); std::exit(4); } \
  } while (0)

static std::vector<char> read_file(const std::string& p, size_t bytes) {
  std::vector<char> b(bytes);
  FILE* f = std::fopen(p.c_str(), "rb");
  if (!f || std::fread(b.data(), 1, bytes, f) != bytes) { std::fprintf(stderr, "cannot read %s\n", p.c_str()); std::exit(2); }
  std::fclose(f);
  return b;
}
static void write_file(const std::string& p, const void* dev, size_t bytes) {
  std::vector<char> b(bytes);
  CHECK_HIP(hipMemcpy(b.data(), dev, bytes, hipMemcpyDeviceToHost));
  FILE* f = std::fopen(p.c_str(), "wb");
  if (!f || std::fwrite(b.data(), 1, bytes, f) != bytes) { std::fprintf(stderr, "cannot write %s\n", p.c_str()); std::exit(2); }
  std::fclose(f);
}
static void* dalloc(size_t bytes) {
  void* p = nullptr;
  CHECK_HIP(hipMalloc(&p, bytes));
  return p;
}

int main(int argc, char** argv) {
  if (argc != 6) { std::fprintf(stderr, "usage: int8_step B H S D dir\n"); return 1; }
  const long B = std::atol(argv[1]), H = std::atol(argv[2]), S = std::atol(argv[3]);
  const int D = std::atoi(argv[4]);
  const std::string dir = argv[5];
  if (qattn_abi_version() != QATTN_ABI_VERSION) {   // a library built against another header
    std::fprintf(stderr, "libqattn ABI %d, this host speaks %d\n", qattn_abi_version(), QATTN_ABI_VERSION);
    return 1;
  }
  const long N = B * H * S;
  const size_t f16b = (size_t)N * D * 2, i8b = (size_t)N * D, sb = (size_t)(N / 32) * 2;
  // the scales of attention_int8.py:151-153 (double products rounded to fp32, as the drop-in does)
  const float qks = (float)(1.0 / std::sqrt((double)D) * 1.44269504);
  const float sms = (float)(1.0 / std::sqrt((double)D));
  hipStream_t st;
  CHECK_HIP(hipStreamCreate(&st));

  void *q = dalloc(f16b), *k = dalloc(f16b), *v = dalloc(f16b), *dO = dalloc(f16b);
  const char* names[4] = {"q", "k", "v", "dO"};
  void* ins[4] = {q, k, v, dO};
  for (int i = 0; i < 4; ++i) {
    const auto h = read_file(dir + "/" + names[i] + ".f16", f16b);
    CHECK_HIP(hipMemcpy(ins[i], h.data(), f16b, hipMemcpyHostToDevice));
  }
  void *q_i8 = dalloc(i8b), *k_i8 = dalloc(i8b), *v_i8 = dalloc(i8b), *vt = dalloc(i8b);
  void *sq = dalloc(sb), *sk = dalloc(sb), *sv = dalloc(sb), *k_mean = dalloc((size_t)B * H * D * 2);
  void *q_bf = dalloc(f16b), *k_bf = dalloc(f16b), *O = dalloc(f16b), *lse = dalloc((size_t)N * 2);
  // forward (attention_int8._int8_forward, smooth=True, images=True, P.V mode i8)
  CHECK_QA(qattn_kmean(k, k_mean, B * H, S, D, st));
  CHECK_QA(qattn_int8_quant_img(q, q_i8, sq, nullptr, q_bf, nullptr, N, (int)S, D, st));
  CHECK_QA(qattn_int8_quant_img(k, k_i8, sk, nullptr, k_bf, k_mean, N, (int)S, D, st));
  CHECK_QA(qattn_int8_quant_vt(v, v_i8, sv, vt, N, D, st));
  CHECK_QA(qattn_int8_attn_fwd_ex(q_i8, sq, k_i8, sk, vt, sv, O, lse, B * H, S, S, 1, 0, D, qks, st));
  // backward (attention_int8._int8_backward: prologue, then the one-pass dS-record backward)
  void *dO_i8 = dalloc(i8b), *sdO = dalloc(sb), *LD = dalloc((size_t)N * 8), *dO_bf = dalloc(f16b);
  void *dq = dalloc(f16b), *dk = dalloc(f16b), *dv = dalloc(f16b);
  CHECK_QA(qattn_int8_bwd_prep(dO, O, lse, dO_i8, sdO, LD, dO_bf, B * H, S, D, st));
  const long ws_bytes = qattn_int8_bwd_ws_bytes(B * H, S, S);
  void* ws = dalloc((size_t)ws_bytes);
  CHECK_QA(qattn_int8_attn_bwd_ws(dO_i8, sdO, q_i8, sq, k_i8, sk, v_i8, sv, LD, q_bf, k_bf, dO_bf, dq, dk,
                                  dv, ws, B * H, S, S, 1, 0, D, qks, sms, st));
  CHECK_HIP(hipStreamSynchronize(st));
  write_file(dir + "/O.f16", O, f16b);
  write_file(dir + "/lse.f16", lse, (size_t)N * 2);
  write_file(dir + "/dq.f16", dq, f16b);
  write_file(dir + "/dk.f16", dk, f16b);
  write_file(dir + "/dv.f16", dv, f16b);
  std::printf("int8_step ok: %ld x %d, workspace %ld B\n", N, D, ws_bytes);
  for (void* p : {q, k, v, dO, q_i8, k_i8, v_i8, vt, sq, sk, sv, k_mean, q_bf, k_bf, O, lse, dO_i8, sdO, LD,
                  dO_bf, dq, dk, dv, ws})
    CHECK_HIP(hipFree(p));
  CHECK_HIP(hipStreamDestroy(st));
  return 0;
}
