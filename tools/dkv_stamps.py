"""Where a fused dK+dV workgroup's time goes (dev tool): the diagnostic build -DQA_DKV_STAMP=1
(tools/ab_build.sh int8_bwd.hip stamp -DQA_DKV_STAMP=1) stamps entry, end of prologue, end of the
tile loop and exit of every workgroup (s_memrealtime, 100 MHz); this runs one config-3 chunk launch
(32 heads, 512 workgroups) and prints the phase durations and the dispatch rounds.

    QATTN_AB=_ab/libqattn_stamp.so python tools/dkv_stamps.py [S] [heads]"""
import ctypes
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd._lib import SIGNATURES  # noqa: E402

torch.cuda.init()
lib = ctypes.CDLL(os.environ["QATTN_AB"], mode=ctypes.RTLD_GLOBAL)
fn = lib.qattn_int8_bwd_dkdv_ws
fn.argtypes = SIGNATURES["qattn_int8_bwd_dkdv_ws"]
S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
bh = int(sys.argv[2]) if len(sys.argv) > 2 else 32
D = 128
N = bh * S
g = torch.Generator(device="cuda").manual_seed(0)
i8 = lambda: torch.randint(-127, 128, (N, D), device="cuda", generator=g, dtype=torch.int8)  # noqa: E731
sc = lambda: (torch.rand(N // 32, device="cuda", generator=g) * 0.01 + 0.01).half()  # noqa: E731
qi, ki, vi, dOi = i8(), i8(), i8(), i8()
sq, sk, sv, sdO = sc(), sc(), sc(), sc()
qb, ob = qi.bfloat16(), dOi.bfloat16()
LD = torch.stack([torch.full((N,), 12.0, device="cuda"), torch.zeros(N, device="cuda")], 1).contiguous()
dk, dv = (torch.empty((N, D), dtype=torch.float16, device="cuda") for _ in range(2))
wsb = ctypes.CDLL(os.environ["QATTN_AB"]).qattn_int8_bwd_ws_bytes
wsb.argtypes = [ctypes.c_long] * 3
wsb.restype = ctypes.c_long
ws = torch.empty((wsb(bh, S, S),), dtype=torch.uint8, device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
sms = float(torch.tensor(1 / math.sqrt(D), dtype=torch.float32))
causal = os.environ.get("CAUSAL") == "1"
if causal:   # the causal record backward in one pass (dK+dV stamped, then dQ from the records)
    full = lib.qattn_int8_attn_bwd_ws
    full.argtypes = SIGNATURES["qattn_int8_attn_bwd_ws"]
    kb = ki.bfloat16()
    dq = torch.empty((N, D), dtype=torch.float16, device="cuda")
for _ in range(int(os.environ.get("REPS", "3"))):   # launches before the stamped (last) one
    if causal:
        rc = full(P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv), P(LD), P(qb), P(kb), P(ob),
                  P(dq), P(dk), P(dv), P(ws), bh, S, S, 1, 1, D, qks, sms, st)
    else:
        rc = fn(P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv), P(LD), P(qb), P(ob), P(dk), P(dv),
                P(ws), bh, S, D, qks, sms, st)
    assert rc == 0
torch.cuda.synchronize()
buf = np.zeros((4096, 4), dtype=np.uint64)
assert lib.qattn_dkv_stamps(ctypes.c_void_p(buf.ctypes.data)) == 0
nwg = bh * S // 256
t = buf[:nwg].astype(np.int64)
t -= t[:, 0].min()
us = t / 100.0   # 100 MHz ticks -> us
pro, loop, epi = us[:, 1] - us[:, 0], us[:, 2] - us[:, 1], us[:, 3] - us[:, 2]
print(f"{nwg} workgroups, kernel span {us[:, 3].max():.1f} us")
for name, x in (("prologue", pro), ("tile loop", loop), ("epilogue", epi), ("start", us[:, 0]),
                ("end", us[:, 3])):
    print(f"  {name:9s} min {x.min():7.1f}  median {np.median(x):7.1f}  max {x.max():7.1f} us")
busy = (us[:, 3] - us[:, 0]).sum()
print(f"  workgroup-time {busy:.0f} us over 256 CUs: {busy / 256:.1f} us per CU if perfectly packed "
      f"({busy / 256 / us[:, 3].max() * 100:.1f} % of the span)")
ends = np.sort(us[:, 3])
print("  last ends (us):", np.round(ends[-8:], 1).tolist(), " 90th pct end", round(float(np.percentile(ends, 90)), 1))
if causal:   # loop time against the workgroup's tile count (bid -> key block as the kernel's grid order)
    nxb = S // 256
    hg = int(os.environ.get("HG", "4"))   # QA_DKV_HG of the build (0: longest-first over all heads)
    bid = np.arange(nwg)
    j = bid >> 3
    if hg > 0 and (bh // 8) % hg == 0:
        r = (j % (hg * nxb)) // hg
    else:
        r = j // (bh // 8)
    ntile = S // 32 - 8 * r
    A = np.vstack([np.ones(nwg), ntile]).T
    coef = np.linalg.lstsq(A, loop, rcond=None)[0]
    print(f"  tile loop ~ {coef[0]:.1f} us + {coef[1]:.3f} us per tile (fit over {nwg} workgroups); "
          f"per-tile time by length: " + " ".join(f"{n}:{np.median(loop[ntile == n]) / n:.2f}" for n in (8, 32, 64, 96, 128)))
order = np.argsort(us[:, 0])
starts = us[order, 0]
print("  start-time histogram (us):", np.histogram(starts, bins=8)[0].tolist(),
      np.round(np.histogram(starts, bins=8)[1], 1).tolist())
# loop time by XCD (bid & 7), by key block (the workgroup's xt under xcd_remap) and by round
bid = np.arange(nwg)
nxb = S // 256
xt = (bid >> 3) % nxb
rnd = (us[:, 0] > us[:, 0].min() + 5).astype(int)
for name, key, n in (("xcd", bid & 7, 8), ("key block", xt, nxb), ("round", rnd, 2)):
    med = [np.median(loop[key == i]) if (key == i).any() else float("nan") for i in range(n)]
    print(f"  loop median by {name}: " + " ".join(f"{m:.1f}" for m in med))
