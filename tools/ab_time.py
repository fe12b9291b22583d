"""Time the int8 attention forward kernel of the library named by QATTN_LIB (A/B dev tool)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_int8 import _int8_forward  # noqa: E402

B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,32,4096,128").split(","))
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
O, lse, qi, kiT, vi, sq, sk, sv, _, _, _ = _int8_forward(q, k, v, False)
N = B * H * S
vdq = torch.empty((N, D), dtype=torch.float16, device="cuda")
st = _lib.stream_of(q)
P = _lib.ptr
_lib.call("qattn_int8_quant", P(v), P(vi), P(sv), P(vdq), None, N, S, D, st)
ki = kiT.t()
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
f = lambda: _lib.call("qattn_int8_attn_fwd", P(qi), P(sq), P(ki), P(sk), P(vdq), P(O), P(lse),  # noqa
                      B * H, S, D, qks, st)
for _ in range(3):
    f()
torch.cuda.synchronize()
ts = []
for _ in range(15):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    f()
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ts.sort()
t = ts[len(ts) // 2]
ops = 4 * B * H * S * S * D
print(f"{os.environ.get('QATTN_LIB', 'default')}: {t * 1e3:.1f} us  {ops / t / 1e9:.0f} TOPS "
      f"({ops / t / 1e9 / 5033 * 100:.1f}% i8 peak)", flush=True)
