"""Diagnostic: time the int8 forward kernel with parts removed (AB=1 no softmax, 2 no PV, 3 no QK)."""
import math, sys, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from quantizedattention_amd import _lib
from quantizedattention_amd.attention_int8 import _int8_forward
B, H, S, D = 4, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
N = B * H * S; P = _lib.ptr; st = _lib.stream_of(q)
O, lse, qi, kiT, vi, sq, sk, sv, km, _, _ = _int8_forward(q, k, v, False)
ki = kiT.t(); vdq = torch.empty((N, D), dtype=torch.float16, device="cuda")
_lib.call("qattn_int8_quant", P(v), P(vi), P(sv), P(vdq), None, N, S, D, st)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
res = {}
for rnd in range(3):
    for ab in (0, 1, 2, 3, 4, 5, 6, 7):
        f = lambda: _lib.call("qattn_int8_attn_fwd_ablate", P(qi), P(sq), P(ki), P(sk), P(vdq), P(O), P(lse), B * H, S, qks, ab, st)
        for _ in range(2): f()
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10): f()
        b.record(); torch.cuda.synchronize()
        res.setdefault(ab, []).append(a.elapsed_time(b) / 10 * 1e3)
for ab, t in res.items():
    names = ['full', 'no-softmax', 'no-PV', 'no-QK', 'no-stream', 'no-stream+no-softmax', 'no-softmax+halfV', 'no-softmax+halfK']
    print(f"AB={ab} ({names[ab]}): {min(t):.1f} us")
