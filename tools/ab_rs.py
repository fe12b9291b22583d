"""Time the role-split int8 forward of ONE library (A/B dev tool, as tools/ab_time.py):
    QATTN_AB=_ab/libqattn_<variant>.so python tools/ab_rs.py [B,H,S,D]"""
import ctypes
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
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
N = B * H * S
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
e = lambda *s, dt: torch.empty(s, dtype=dt, device="cuda")  # noqa: E731
qi, ki, vi = (e(N, D, dt=torch.int8) for _ in range(3))
sq, sk, sv = (e(N // 32, dt=torch.float16) for _ in range(3))
vop = e(N, D, dt=torch.float16)
O, lse = e(N, D, dt=torch.float16), e(N, dt=torch.float16)
call("qattn_int8_quant", P(q), P(qi), P(sq), None, None, N, S, D, st)
call("qattn_int8_quant", P(k), P(ki), P(sk), None, None, N, S, D, st)
call("qattn_int8_quant_vop", P(v), P(vi), P(sv), P(vop), N, D, st)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
fn = lambda: call("qattn_int8_attn_fwd_rs", P(qi), P(sq), P(ki), P(sk), P(vop), P(O), P(lse),  # noqa: E731
                  B * H, S, S, 1, D, qks, st)
for _ in range(3):
    fn()
ts = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10 * 1e3)
print(f"{os.path.basename(path)}: rs {' '.join(f'{t:.0f}' for t in ts)} us", flush=True)
