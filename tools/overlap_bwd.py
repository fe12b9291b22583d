"""Does the dQ-from-records pass of chunk c overlap the dK+dV pass of chunk c+1 on a second stream?
(dev tool; config 3, chunks of 32 heads as the step runs them).  Sequential: dK+dV(c), dQ(c) on one
stream with one workspace (qattn_int8_attn_bwd_wsc).  Overlapped: two workspaces; dQ(c) on a side
stream after dK+dV(c), dK+dV(c+2) after dQ(c) (workspace reuse).  Prints both times and whether
dq / dk / dv are bit-identical.

    python tools/overlap_bwd.py"""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_int8 import _int8_forward, _ws_chunk  # noqa: E402

B, H, S, D = 4, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
O, lse, qi, kiT, vi, sq, sk, sv, km, qb, kb = _int8_forward(q, k, v, smooth=True, images=True)
ki = kiT.t().contiguous()
N, BH = B * H * S, B * H
P = _lib.ptr
main = torch.cuda.current_stream()
st = _lib.stream_of(O)
dOi = torch.empty((N, D), dtype=torch.int8, device="cuda")
sdO = torch.empty((N // 32,), dtype=torch.float16, device="cuda")
LD = torch.empty((N, 2), dtype=torch.float32, device="cuda")
dOb = torch.empty((N, D), dtype=torch.bfloat16, device="cuda")
_lib.call("qattn_int8_bwd_prep", P(dO), P(O), P(lse), P(dOi), P(sdO), P(LD), P(dOb), BH, S, D, st)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
sms = float(torch.tensor(1 / math.sqrt(D), dtype=torch.float32))
chunk = _ws_chunk(None, False, BH, S)
wsb = _lib.load().qattn_int8_bwd_ws_bytes(chunk, S, S)
ws = [torch.empty((wsb,), dtype=torch.uint8, device="cuda") for _ in range(2)]
qf, kf, vf, qbf, kbf = qi.view(N, D), ki.view(N, D), vi.view(N, D), qb.view(N, D), kb.view(N, D)
outs = {}


def dkdv(c, w, dq, dk, dv, s):
    r = slice(c * chunk * S, (c + 1) * chunk * S)
    b = slice(c * chunk * S // 32, (c + 1) * chunk * S // 32)
    _lib.call("qattn_int8_bwd_dkdv_ws", P(dOi[r]), P(sdO[b]), P(qf[r]), P(sq[b]), P(kf[r]), P(sk[b]),
              P(vf[r]), P(sv[b]), P(LD[r]), P(qbf[r]), P(dOb[r]), P(dk[r]), P(dv[r]), P(w), chunk, S,
              D, qks, sms, s)


def dqw(c, w, dq, s):
    r = slice(c * chunk * S, (c + 1) * chunk * S)
    b = slice(c * chunk * S // 32, (c + 1) * chunk * S // 32)
    _lib.call("qattn_int8_bwd_dq_ws", P(kbf[r]), P(sk[b]), P(dq[r]), P(w), chunk, S, D, sms, s)


nch = BH // chunk
side = torch.cuda.Stream()
side_st = ctypes.c_void_p(side.cuda_stream)


def sequential(dq, dk, dv):
    for c in range(nch):
        dkdv(c, ws[0], dq, dk, dv, st)
        dqw(c, ws[0], dq, st)


def overlapped(dq, dk, dv):
    ev_a = [torch.cuda.Event() for _ in range(nch)]
    ev_b = [torch.cuda.Event() for _ in range(nch)]
    side.wait_stream(main)
    for c in range(nch):
        if c >= 2:
            main.wait_event(ev_b[c - 2])
        dkdv(c, ws[c % 2], dq, dk, dv, st)
        ev_a[c].record(main)
        side.wait_event(ev_a[c])
        dqw(c, ws[c % 2], dq, side_st)
        ev_b[c].record(side)
    main.wait_stream(side)


def run(fn, name, reps=10):
    dq, dk, dv = (torch.empty((N, D), dtype=torch.float16, device="cuda") for _ in range(3))
    for _ in range(2):
        fn(dq, dk, dv)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        fn(dq, dk, dv)
        b.record(main)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    outs[name] = (dq, dk, dv)
    print(f"{name}: {ts[len(ts) // 2]:.1f} us (min {ts[0]:.1f}, max {ts[-1]:.1f})", flush=True)


run(sequential, "sequential")
run(overlapped, "overlapped")
run(sequential, "sequential")
run(overlapped, "overlapped")
same = all(torch.equal(a, b) for a, b in zip(outs["sequential"], outs["overlapped"]))
print("dq/dk/dv bit-identical:", same)
