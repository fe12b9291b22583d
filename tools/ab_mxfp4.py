"""Time the MX-FP4 forward kernel and its quantisers (dev tool).

    python tools/ab_mxfp4.py [B,H,S,D]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_mxfp4 import (mxfp4_attn_fwd, mxfp4_quantize_rows,  # noqa: E402
                                                    mxfp4_quantize_v)

B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,32,4096,128").split(","))
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
k = torch.randn((B, H, S, D), device="cuda", generator=g).half()
v = torch.randn((B, H, S, D), device="cuda", generator=g).half()
O, lse, (q4, qs, k4, ks, vt, vs) = mxfp4_attn_fwd(q, k, v)
qks = float(torch.tensor(1.0 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
st = _lib.stream_of(q)


def kernel():
    _lib.call("qattn_mxfp4_attn_fwd", _lib.ptr(q4), _lib.ptr(qs), _lib.ptr(k4), _lib.ptr(ks), _lib.ptr(vt),
              _lib.ptr(vs), _lib.ptr(O), _lib.ptr(lse), B * H, S, S, 1, D, qks, st)


def timed(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


tk = timed(kernel)
tq = timed(lambda: (mxfp4_quantize_rows(q), mxfp4_quantize_rows(k), mxfp4_quantize_v(v)))
te = timed(lambda: mxfp4_attn_fwd(q, k, v))
flop = 4 * B * H * S * S * D
print(f"{os.environ.get('QATTN_LIB', 'default')}: mxfp4 fwd kernel {tk * 1e3:.1f} us = {flop / tk / 1e9:.0f} TFLOP/s "
      f"({flop / tk / 1e9 / 10066 * 100:.1f}% of the 10.07 PF dense fp4 peak); "
      f"quantisers {tq * 1e3:.1f} us; end-to-end {te * 1e3:.1f} us", flush=True)
