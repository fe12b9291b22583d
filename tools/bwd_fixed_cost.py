"""Per-workgroup fixed cost of the record backward (dev tool): dK+dV with records and dQ from the
records at a constant 512 dK+dV workgroups (bh = 512 * 256 / S heads) for S = 1024, 2048, 4096 --
tiles per workgroup S / 32 -- and the fit time = tiles * T + F per launch.

    python tools/bwd_fixed_cost.py"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd import _lib  # noqa: E402

D = 128
g = torch.Generator(device="cuda").manual_seed(0)
st = _lib.stream_of(torch.empty(1, device="cuda"))
P = _lib.ptr
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
sms = float(torch.tensor(1 / math.sqrt(D), dtype=torch.float32))


def time_it(f, reps=8):
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


res = {"dkdv": [], "dqw": []}
for S in (1024, 2048, 4096):
    bh = 512 * 256 // S
    N = bh * S
    i8 = lambda: torch.randint(-127, 128, (N, D), device="cuda", generator=g, dtype=torch.int8)  # noqa: E731
    sc = lambda: (torch.rand(N // 32, device="cuda", generator=g) * 0.01 + 0.01).half()  # noqa: E731
    qi, ki, vi, dOi = i8(), i8(), i8(), i8()
    sq, sk, sv, sdO = sc(), sc(), sc(), sc()
    qb, kb, ob = (t.bfloat16() for t in (qi, ki, dOi))
    LD = torch.stack([torch.full((N,), 12.0, device="cuda"), torch.zeros(N, device="cuda")], 1).contiguous()
    dq, dk, dv = (torch.empty((N, D), dtype=torch.float16, device="cuda") for _ in range(3))
    ws = torch.empty(_lib.load().qattn_int8_bwd_ws_bytes(bh, S, S), dtype=torch.uint8, device="cuda")
    f1 = lambda: _lib.call("qattn_int8_bwd_dkdv_ws", P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi),  # noqa: E731
                           P(sv), P(LD), P(qb), P(ob), P(dk), P(dv), P(ws), bh, S, D, qks, sms, st)
    f2 = lambda: _lib.call("qattn_int8_bwd_dq_ws", P(kb), P(sk), P(dq), P(ws), bh, S, D, sms, st)  # noqa: E731
    t1, t2 = time_it(f1), time_it(f2)
    res["dkdv"].append((S // 32, t1))
    res["dqw"].append((S // 32, t2))
    print(f"S {S} bh {bh}: {S // 32} tiles per workgroup: dK+dV {t1:.1f} us, dQ from records {t2:.1f} us",
          flush=True)
    del qi, ki, vi, dOi, qb, kb, ob, ws, dq, dk, dv
for k, rows in res.items():
    n = len(rows)
    sx = sum(r[0] for r in rows); sy = sum(r[1] for r in rows)
    sxx = sum(r[0] ** 2 for r in rows); sxy = sum(r[0] * r[1] for r in rows)
    a = (n * sxy - sx * sy) / (n * sxx - sx ** 2)
    b = (sy - a * sx) / n
    print(f"{k}: {a:.3f} us per tile-column + {b:.1f} us fixed per launch")
