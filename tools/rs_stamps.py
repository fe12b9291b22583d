"""Phase timeline of the role-split forward from a diagnostic build (-DQA_RS_STAMP=1): s_memtime
stamps of steps 40..47 of workgroup 777 (matrix wave 0, softmax wave NM).  Dev tool:
    QATTN_AB=_ab/libqattn_<stamp variant>.so python tools/rs_stamps.py"""
import ctypes
import os
import runpy
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.argv = [sys.argv[0]]
g = runpy.run_path(os.path.join(ROOT, "tools", "ab_rs.py"))   # runs the kernel (loads QATTN_AB)
lib = g["lib"]
buf = np.zeros((2, 8, 16), dtype=np.uint64)
lib.qattn_rs_stamps.argtypes = [ctypes.c_void_p]
assert lib.qattn_rs_stamps(buf.ctypes.data) == 0
m, v = buf[0].astype(np.int64), buf[1].astype(np.int64)
t0 = m[0, 0]
print("matrix wave: step start, +QK issued, +P/r read, +PV issued, +S written, +prefetch/DMA issued, +vmcnt ok")
for s in range(8):
    r = m[s, :7] - t0
    print(f"  step {40 + s}: " + " ".join(f"{x:7d}" for x in r), "  d:", " ".join(f"{x:5d}" for x in np.diff(r)))
print("softmax wave: tile start, +row max, +P ready, +sm done, +lgkm, +barrier out")
for s in range(8):
    r = v[s, :6] - t0
    print(f"  step {40 + s}: " + " ".join(f"{x:7d}" for x in r), "  d:", " ".join(f"{x:5d}" for x in np.diff(r)))
