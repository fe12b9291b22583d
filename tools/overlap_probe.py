"""Does a CU-based copy overlap the int8 backward?  (Proxy for RCCL's CU kernels during dK+dV at
config 4, SURVEY §8e: each rank receives 470 MB of O.)  Dev tool:
    python tools/overlap_probe.py [chunks] [add | memcpy | few<N>]
add: a grid-filling elementwise kernel; memcpy: hipMemcpyAsync D2D; few<N>: a copy kernel of exactly
N workgroups (as an RCCL collective moves its bytes with a few persistent workgroups).

Times, HIP events on the compute stream: the config-3 int8 backward alone; a 470 MB device copy
(an elementwise CU kernel, out = src + 0) alone on a side stream; both launched together.  If the
pair takes about the sum, the copy is starved while the backward holds the CUs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward  # noqa: E402

torch.cuda.init()
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((4, 32, 4096, 128), device="cuda", generator=g).half() for _ in range(3))
dO = (torch.randn((4, 32, 4096, 128), device="cuda", generator=g) * 1e-3).half()
O, lse, qi, kiT, vi, sq, sk, sv, km, qb, kb = _int8_forward(q, k, v, smooth=True, images=True)
n = 470_000_000 // 2
src = torch.randn(n, device="cuda", generator=g).half()
dst = torch.empty_like(src)
side = torch.cuda.Stream()
chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 1


def bwd():
    _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb)


MODE = sys.argv[2] if len(sys.argv) > 2 else "add"


def copy():
    step = (n + chunks - 1) // chunks
    for c in range(chunks):
        if MODE == "add":      # an elementwise CU kernel
            torch.add(src[c * step:(c + 1) * step], 0, out=dst[c * step:(c + 1) * step])
        elif MODE.startswith("few"):   # a copy kernel of a fixed, small number of workgroups
            a, b = src[c * step:(c + 1) * step], dst[c * step:(c + 1) * step]
            _lib.call("qattn_probe_few_wg_copy", _lib.ptr(a), _lib.ptr(b), a.numel() * 2,
                      int(MODE[3:]), _lib.stream_of(b))
        else:                  # hipMemcpyAsync device-to-device (the runtime picks blit kernel or SDMA)
            dst[c * step:(c + 1) * step].copy_(src[c * step:(c + 1) * step])


def t(fn, stream=None, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s = stream or torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def both():
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        copy()
    bwd()
    torch.cuda.current_stream().wait_stream(side)


tb, tc, tt = t(bwd), t(copy, side), t(both)
print(f"[{MODE}, {chunks} chunk(s)] backward {tb:.3f} ms | copy 470 MB {tc:.3f} ms ({470e6 / tc / 1e9:.2f} TB/s) | "
      f"together {tt:.3f} ms "
      f"(sum {tb + tc:.3f}, overlap hides {(tb + tc - tt) / tc * 100:.0f}% of the copy)", flush=True)
