"""Per-workgroup fixed cost of the int8 forward (dev tool): time the non-causal kernel at Sq = 4096
against Sk = 128 .. 4096 keys (same grid, tiles per workgroup = Sk / 32) and fit time = rounds *
(tiles * T + F); also the causal kernel at the same shape for comparison.

    python tools/fwd_fixed_cost.py"""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd import _lib  # noqa: E402

B, H, Sq, D = 4, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
N = B * H * Sq
qi = torch.randint(-127, 128, (N, D), device="cuda", generator=g, dtype=torch.int8)
sq = (torch.rand(N // 32, device="cuda", generator=g) * 0.01 + 0.01).half()
O = torch.empty((N, D), dtype=torch.float16, device="cuda")
lse = torch.empty((N,), dtype=torch.float16, device="cuda")
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
st = _lib.stream_of(O)


def time_it(f, reps=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


rows = []
for Sk in (128, 256, 512, 1024, 2048, 4096):
    Nk = B * H * Sk
    ki = torch.randint(-127, 128, (Nk, D), device="cuda", generator=g, dtype=torch.int8)
    vt = torch.randint(-127, 128, (Nk, D), device="cuda", generator=g, dtype=torch.int8)
    sk = (torch.rand(Nk // 32, device="cuda", generator=g) * 0.01 + 0.01).half()
    sv = (torch.rand(Nk // 32, device="cuda", generator=g) * 0.01 + 0.01).half()
    P = _lib.ptr

    def f(causal=0):
        _lib.call("qattn_int8_attn_fwd_ex", P(qi), P(sq), P(ki), P(sk), P(vt), P(sv), P(O), P(lse),
                  B * H, Sq, Sk, 1, causal, D, qks, st)
    t = time_it(f)
    rows.append((Sk // 32, t))
    print(f"Sk {Sk:5d} ({Sk // 32:3d} tiles per workgroup): {t:8.1f} us", flush=True)
    if Sk == 4096:
        print(f"causal Sk {Sk}: {time_it(lambda: f(1)):8.1f} us", flush=True)
# least squares t = a * tiles + b
n = len(rows)
sx = sum(r[0] for r in rows); sy = sum(r[1] for r in rows)
sxx = sum(r[0] ** 2 for r in rows); sxy = sum(r[0] * r[1] for r in rows)
a = (n * sxy - sx * sy) / (n * sxx - sx ** 2)
b = (sy - a * sx) / n
print(f"fit: {a:.3f} us per tile-column + {b:.1f} us fixed (8 rounds of 512 workgroups: "
      f"{b / 8:.2f} us per workgroup)")
