"""Time the HBM-bound int8 passes of the step (k-mean, the quantisers with their bf16 images, the
V^T image, the backward prologue) of one library, and hash their outputs so that two builds can be
compared bit for bit (A/B dev tool: tools/ab_build.sh builds variants).

    QATTN_AB=_ab/libqattn_<variant>.so python tools/ab_quant.py [B,H,S,D]

One library per process (see tools/ab_time.py)."""
import ctypes
import hashlib
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd._lib import SIGNATURES  # noqa: E402

path = os.environ.get("QATTN_AB") or os.path.join(ROOT, "quantizedattention_amd", "libqattn.so")
torch.cuda.init()
lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def call(name, *args):
    fn = getattr(lib, name)
    fn.argtypes = SIGNATURES[name]
    fn.restype = ctypes.c_int
    rc = fn(*args)
    assert rc == 0, (name, rc)


B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,32,4096,128").split(","))
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v, O = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(4))
dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
lse = torch.randn((B * H * S,), device="cuda", generator=g).half()
N = B * H * S
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
e = lambda *s, dt: torch.empty(s, dtype=dt, device="cuda")  # noqa: E731
km = e(B * H, D, dt=torch.float16)
qi, ki, vi, vt, di = (e(N, D, dt=torch.int8) for _ in range(5))
sq, sk, sv, sd = (e(N // 32, dt=torch.float16) for _ in range(4))
qb, kb, db = (e(N, D, dt=torch.bfloat16) for _ in range(3))
LD = e(N, 2, dt=torch.float32)
fns = {
    "kmean": lambda: call("qattn_kmean", P(k), P(km), B * H, S, D, st),
    "quant_img(q)": lambda: call("qattn_int8_quant_img", P(q), P(qi), P(sq), None, P(qb), None, N, S, D, st),
    "quant_img(k, smooth)": lambda: call("qattn_int8_quant_img", P(k), P(ki), P(sk), None, P(kb), P(km),
                                         N, S, D, st),
    "quant_vt(v)": lambda: call("qattn_int8_quant_vt", P(v), P(vi), P(sv), P(vt), N, D, st),
    "quant(k, smooth, no img)": lambda: call("qattn_int8_quant_img", P(k), P(ki), P(sk), None, None, P(km),
                                             N, S, D, st),
    "kmean+quant(k) 2 launches": lambda: (call("qattn_kmean", P(k), P(km), B * H, S, D, st),
                                          call("qattn_int8_quant_img", P(k), P(ki), P(sk), None, None, P(km),
                                               N, S, D, st)),
    "k_smooth fused": lambda: call("qattn_int8_quant_k_smooth", P(k), P(km), P(ki), P(sk), None, B * H, S, D,
                                   st),
    "k_smooth fused +img": lambda: call("qattn_int8_quant_k_smooth", P(k), P(km), P(ki), P(sk), P(kb), B * H,
                                        S, D, st),
    "bwd_prep": lambda: call("qattn_int8_bwd_prep", P(dO), P(O), P(lse), P(di), P(sd), P(LD), P(db),
                             B * H, S, D, st),
}
bytes_of = {"kmean": N * D * 2, "quant_img(q)": N * D * 5, "quant_img(k, smooth)": N * D * 5,
            "quant_vt(v)": N * D * 4, "bwd_prep": N * D * 7 + N * 10, "quant(k, smooth, no img)": N * D * 3,
            "kmean+quant(k) 2 launches": N * D * 5, "k_smooth fused": N * D * 3, "k_smooth fused +img": N * D * 5}
if getattr(lib, "qattn_int8_quant_k_smooth", None) is None:   # (an older library)
    for n_ in ("k_smooth fused", "k_smooth fused +img"):
        fns.pop(n_)
res = {}
for name, f in fns.items():
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    res[name] = ts[len(ts) // 2]
h = hashlib.sha256()
for t in (km, qi, ki, vi, vt, di, sq, sk, sv, sd, qb, kb, db, LD):
    h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
print(os.path.basename(path), " | ".join(f"{n} {us:.1f} us ({bytes_of[n] / us / 1e6:.2f} TB/s)"
                                         for n, us in res.items()), "| outputs", h.hexdigest()[:16],
      flush=True)
