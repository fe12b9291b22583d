"""Causal int8 backward at config 3 by chunk size (dev tool): QATTN_BWD_WS_CHUNK=<kv heads per chunk>
python tools/ab_causal_chunk.py  -> median ms of _int8_backward(causal=True) and an output digest
(AB_CAUSAL=0: the non-causal backward)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
B, H, S, D = 4, 32, 4096, 128
causal = os.environ.get("AB_CAUSAL", "1") == "1"
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
O, lse, qi, kiT, vi, sq, sk, sv, km, qb, kb = _int8_forward(q, k, v, smooth=True, images=True, causal=causal)
f = lambda: _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, causal=causal)  # noqa: E731
for _ in range(2):
    out = f()
torch.cuda.synchronize()
ts = []
for _ in range(7):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    out = f()
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
h = hashlib.sha256()
for x in out[:3]:
    h.update(x.contiguous().view(torch.int16).cpu().numpy().tobytes())
print(f"chunk={os.environ.get('QATTN_BWD_WS_CHUNK', 'auto')}: {'causal' if causal else 'non-causal'} backward {sorted(ts)[3]:.3f} ms, "
      f"grads {h.hexdigest()[:12]}", flush=True)
