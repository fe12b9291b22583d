"""Per-phase cycle breakdown of the int8 forward loop from a QA_FWD_STAMP build (dev tool).
    QATTN_LIB=_ab/libqattn_stamp.so python tools/stamps.py"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_int8 import _int8_forward  # noqa: E402

B, H, S, D = 4, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
O, lse, qi, kiT, vi, sq, sk, sv, _, _, _ = _int8_forward(q, k, v, False)
N = B * H * S
vdq = torch.empty((N, D), dtype=torch.float16, device="cuda")
st = _lib.stream_of(q)
P = _lib.ptr
_lib.call("qattn_int8_quant", P(v), P(vi), P(sv), P(vdq), None, N, S, D, st)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
for _ in range(3):
    O.zero_()
    _lib.call("qattn_int8_attn_fwd", P(qi), P(sq), P(kiT.t()), P(sk), P(vdq), P(O), P(lse), B * H, S, D,
              qks, st)
torch.cuda.synchronize()
import ctypes  # noqa: E402
import numpy as np  # noqa: E402
stamps = np.zeros(32 * 4 * 64 * 8, dtype=np.int64)
wginfo = np.zeros(8192 * 4, dtype=np.int64)
_lib.load().qattn_fwd_stamps(ctypes.c_void_p(stamps.ctypes.data), ctypes.c_void_p(wginfo.ctypes.data))
st64 = torch.from_numpy(stamps).view(32 * 4, 64, 8)
names = ["barrier", "dma+sk+pv_load+qk", "sm2", "pv_mma", "sm1a", "sm1b", "->next"]
d = []
for kk in range(6):
    d.append((st64[:, 8:60, kk + 1] - st64[:, 8:60, kk]).float())
d.append((st64[:, 9:61, 0] - st64[:, 8:60, 6]).float())
tot = (st64[:, 9:61, 0] - st64[:, 8:60, 0]).float()
for n, x in zip(names, d):
    print(f"{n:22s} mean {x.mean():8.1f}  median {x.median():8.1f}")
print(f"{'tile total':22s} mean {tot.mean():8.1f}  median {tot.median():8.1f}")

# ---- residency: workgroups per CU over time (per XCD clock domain)
w = torch.from_numpy(wginfo)[: 4096 * 4].view(4096, 4)
t0, t1, hw, xcc = w[:, 0], w[:, 1], w[:, 2], w[:, 3] & 0xF
cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
life = (t1 - t0).float()
print("workgroup lifetime: mean %.0f  min %.0f  max %.0f cycles" % (life.mean(), life.min(), life.max()))
conc = []
for kk in key.unique()[:64].tolist():
    m = key == kk
    a, b = t0[m], t1[m]
    ev = sorted([(int(x), 1) for x in a] + [(int(x), -1) for x in b])
    c = mx = 0
    busy = 0
    last = ev[0][0]
    area = 0
    for tt, dlt in ev:
        area += c * (tt - last)
        last = tt
        c += dlt
        mx = max(mx, c)
    span = ev[-1][0] - ev[0][0]
    conc.append((mx, area / span, int(m.sum())))
print("per-CU max resident WGs / mean resident / WGs:", conc[:12])
print("mean resident over CUs: %.2f" % (sum(c[1] for c in conc) / len(conc)))
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"xcc {x}: WGs {int(m.sum())}  span {int(t1[m].max() - t0[m].min())} ticks  "
              f"first start {int(t0[m].min())}")
