"""bf16 causal forward: the V-suffix path (qattn_bf16_fwd_ws_ex) against the full masked tile loop
(qattn_bf16_fwd_ex) in one process: median event times and the largest output differences.

    python tools/ab_bf16_sfx.py [B,H,S,D]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd import _lib  # noqa: E402

B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,32,4096,128").split(","))
lib = _lib.load()
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
k = torch.randn((B, H, S, D), device="cuda", generator=g).half()
v = torch.randn((B, H, S, D), device="cuda", generator=g).bfloat16()
qks = float(torch.tensor(1.0 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
ws = torch.empty(lib.qattn_bf16_fwd_ws_bytes(B * H, S, D) // 4, device="cuda")
res = {}
for name in ("tile_loop", "vsuffix"):
    O = torch.empty((B, H, S, D), device="cuda")
    lse = torch.empty((B * H, S), device="cuda")
    base = (_lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(O), _lib.ptr(lse), B * H, S, S, 1, 1, D, qks)
    st = _lib.stream_of(q)
    f = ((lambda: _lib.call("qattn_bf16_fwd_ex", *base, st)) if name == "tile_loop"
         else (lambda: _lib.call("qattn_bf16_fwd_ws_ex", *base, _lib.ptr(ws), st)))
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
    res[name] = (O, lse, ts[len(ts) // 2])
    print(f"{name}: {ts[len(ts) // 2] * 1e3:.1f} us (min {ts[0] * 1e3:.1f})", flush=True)
(O0, l0, _), (O1, l1, _) = res["tile_loop"], res["vsuffix"]
print(f"max |dO| {(O1 - O0).abs().max().item():.3e}  max |dlse| {(l1 - l0).abs().max().item():.3e}  "
      f"finite {bool(torch.isfinite(O1).all() and torch.isfinite(l1).all())}", flush=True)
