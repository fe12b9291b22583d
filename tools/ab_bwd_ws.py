"""Time one config-3 chunk launch of the record backward (32 heads: dK+dV with records, then dQ
from them) of ONE library, and hash dk / dv / dq so that two builds can be compared bit for bit
(A/B dev tool):  QATTN_AB=_ab/libqattn_<variant>.so python tools/ab_bwd_ws.py"""
import ctypes
import hashlib
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd._lib import SIGNATURES  # noqa: E402

path = os.environ.get("QATTN_AB") or os.path.join(ROOT, "quantizedattention_amd", "libqattn.so")
torch.cuda.init()
lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
for n in ("qattn_int8_bwd_dkdv_ws", "qattn_int8_bwd_dq_ws", "qattn_int8_bwd_ws_bytes"):
    getattr(lib, n).argtypes = SIGNATURES[n]
lib.qattn_int8_bwd_ws_bytes.restype = ctypes.c_long
bh, S, D = int(os.environ.get("BH", "32")), 4096, 128
N = bh * S
g = torch.Generator(device="cuda").manual_seed(0)
i8 = lambda: torch.randint(-127, 128, (N, D), device="cuda", generator=g, dtype=torch.int8)  # noqa: E731
sc = lambda: (torch.rand(N // 32, device="cuda", generator=g) * 0.01 + 0.01).half()  # noqa: E731
qi, ki, vi, dOi = i8(), i8(), i8(), i8()
sq, sk, sv, sdO = sc(), sc(), sc(), sc()
qb, kb, ob = qi.bfloat16(), ki.bfloat16(), dOi.bfloat16()
LD = torch.stack([torch.full((N,), 12.0, device="cuda"), torch.zeros(N, device="cuda")], 1).contiguous()
dq, dk, dv = (torch.empty((N, D), dtype=torch.float16, device="cuda") for _ in range(3))
ws = torch.empty((lib.qattn_int8_bwd_ws_bytes(bh, S, S),), dtype=torch.uint8, device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
sms = float(torch.tensor(1 / math.sqrt(D), dtype=torch.float32))
f1 = lambda: lib.qattn_int8_bwd_dkdv_ws(P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv),  # noqa: E731
                                        P(LD), P(qb), P(ob), P(dk), P(dv), P(ws), bh, S, D, qks, sms, st)
f2 = lambda: lib.qattn_int8_bwd_dq_ws(P(kb), P(sk), P(dq), P(ws), bh, S, D, sms, st)  # noqa: E731


def t(f, reps=15):
    for _ in range(3):
        assert f() == 0
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[reps // 2]


causal = os.environ.get("QATTN_AB_CAUSAL") == "1"
if causal:   # the whole record backward, causal (dK+dV then dQ in one call)
    lib.qattn_int8_attn_bwd_ws.argtypes = SIGNATURES["qattn_int8_attn_bwd_ws"]
    f1 = lambda: lib.qattn_int8_attn_bwd_ws(P(dOi), P(sdO), P(qi), P(sq), P(ki), P(sk), P(vi), P(sv),  # noqa: E731
                                            P(LD), P(qb), P(kb), P(ob), P(dq), P(dk), P(dv), P(ws), bh,
                                            S, S, 1, 1, D, qks, sms, st)
    f2 = lambda: 0  # noqa: E731
t1, t2 = t(f1), t(f2)
if os.environ.get("QATTN_AB_SAVE"):   # outputs for a numeric comparison across builds
    torch.save({"dk": dk.cpu(), "dv": dv.cpu(), "dq": dq.cpu()}, os.environ["QATTN_AB_SAVE"])
if os.environ.get("QATTN_AB_REF"):
    ref = torch.load(os.environ["QATTN_AB_REF"], weights_only=True)
    for n_, x in (("dk", dk), ("dv", dv), ("dq", dq)):
        r = ref[n_].float()
        d = (x.cpu().float() - r).abs()
        print(f"  {n_}: max|diff| {d.max().item():.3g} (max|ref| {r.abs().max().item():.3g}), "
              f"identical {bool(torch.equal(x.cpu(), ref[n_]))}", flush=True)
h = hashlib.sha256()
for x in (dk, dv, dq):
    h.update(x.view(torch.int16).cpu().numpy().tobytes())
print(f"{os.path.basename(path)}{' causal' if causal else ''}: dK+dV {t1:.1f} us, dQ from records {t2:.1f} us, outputs "
      f"{h.hexdigest()[:12]}", flush=True)
