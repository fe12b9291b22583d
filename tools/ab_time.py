"""Time the int8 attention forward kernel of one library (A/B dev tool:
tools/ab_build.sh builds variants, tools/ab_run.sh runs this over them).

    QATTN_AB=_ab/libqattn_<variant>.so python tools/ab_time.py [B,H,S,D] [causal]

Exactly ONE library is loaded per process (the variant, or the in-tree build): two copies of the
same kernels in one process bind each other's identically named template kernel stubs (ELF symbol
interposition), so a variant would launch the other library's code.  The library is bound here with
ctypes directly; entries a variant lacks (an older kernel) are skipped."""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizedattention_amd._lib import SIGNATURES  # noqa: E402  (argtypes only; loads nothing)

path = os.environ.get("QATTN_AB") or os.path.join(ROOT, "quantizedattention_amd", "libqattn.so")
torch.cuda.init()
lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def entry(name):
    fn = getattr(lib, name, None)
    if fn is not None:
        fn.argtypes = SIGNATURES[name]
        fn.restype = ctypes.c_int
    return fn


def call(name, *args):
    rc = entry(name)(*args)
    assert rc == 0, (name, rc)


B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,32,4096,128").split(","))
causal = len(sys.argv) > 2 and sys.argv[2] == "causal"
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
N = B * H * S
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
e = lambda *s, dt: torch.empty(s, dtype=dt, device="cuda")  # noqa: E731
qi, ki, vi = (e(N, D, dt=torch.int8) for _ in range(3))
sq, sk, sv = (e(N // 32, dt=torch.float16) for _ in range(3))
vt = e(N, D, dt=torch.int8)
O, lse = e(N, D, dt=torch.float16), e(N, dt=torch.float16)
call("qattn_int8_quant", P(q), P(qi), P(sq), None, None, N, S, D, st)
call("qattn_int8_quant", P(k), P(ki), P(sk), None, None, N, S, D, st)
call("qattn_int8_quant_vt", P(v), P(vi), P(sv), P(vt), N, D, st)
qks = float(torch.tensor(1 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
fns = {"i8": lambda: call("qattn_int8_attn_fwd_ex", P(qi), P(sq), P(ki), P(sk), P(vt), P(sv),
                         P(O), P(lse), B * H, S, S, 1, int(causal), D, qks, st)}
if getattr(lib, "qattn_int8_attn_fwd_qf", None) is not None:   # q quantised in the kernel
    qi2, sq2 = e(N, D, dt=torch.int8), e(N // 32, dt=torch.float16)
    fns["qf"] = lambda: call("qattn_int8_attn_fwd_qf", P(q), P(qi2), P(sq2), None, P(ki), P(sk), P(vt),
                             P(sv), P(O), P(lse), B * H, S, S, 1, int(causal), D, qks, st)
only = os.environ.get("QATTN_AB_MODES")
if only:
    fns = {k_: f_ for k_, f_ in fns.items() if k_ in only.split(",")}
ops = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
name = os.path.basename(path)
for mode, f in fns.items():
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
    t = ts[len(ts) // 2]
    if os.environ.get("QATTN_AB_SAVE"):   # O and lse of the last mode timed, for a bitwise diff
        torch.save({"O": O.cpu(), "lse": lse.cpu()}, os.environ["QATTN_AB_SAVE"])
    import hashlib
    digest = hashlib.sha256(O.view(torch.int16).cpu().numpy().tobytes() +
                            lse.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:12]
    ref_o = globals().setdefault("_ref_o", {})
    if not ref_o:
        ref_o["o"], ref_o["l"], ref_o["m"] = O.float().clone(), lse.float().clone(), mode
    dO = (O.float() - ref_o["o"]).abs().max().item()
    dl = (lse.float() - ref_o["l"]).abs().max().item()
    print(f"  max|O - O[{ref_o['m']}]| = {dO:.3g}, max|lse - lse[{ref_o['m']}]| = {dl:.3g}")
    print(f"{name} pv={mode}{' causal' if causal else ''}: {t * 1e3:.1f} us  {ops / t / 1e9:.0f} TOPS "
          f"({ops / t / 1e9 / 5033 * 100:.1f}% i8 peak)  O/lse {digest}", flush=True)
    cnt = getattr(lib, "qattn_fwd_lit_count", None)
    if cnt is not None:   # -DQA_FWD_LIT_COUNT=1 builds: literal tiles per wave-tile since load
        import numpy as np
        buf = np.zeros(4, dtype=np.uint64)
        cnt.argtypes = [ctypes.c_void_p]
        cnt(buf.ctypes.data)
        print(f"  literal wave-tiles {int(buf[0])} of {int(buf[1])} ({100 * buf[0] / max(1, buf[1]):.2f} %), "
              f"waves marked for the fixup {int(buf[2])} of {int(buf[3])} ({100 * buf[2] / max(1, buf[3]):.3f} %)")
