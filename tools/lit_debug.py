"""Parity of the int8 forward against the oracle on the fuzz cases of tests/test_gpu_fuzz.py, per
library (A/B dev tool: QATTN_LIB=_ab/libqattn_<variant>.so python tools/lit_debug.py [case ...])."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import restate as R  # noqa: E402
from test_gpu_fuzz import _case  # noqa: E402
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd  # noqa: E402

cases = [int(c) for c in sys.argv[1:]] or list(range(24))
lib = os.path.basename(os.environ.get("QATTN_LIB", "libqattn.so"))
for i in cases:
    q, k, v, causal = _case(i)
    out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda(), causal=causal)
    ref = R.int8_fwd(q, k, v, causal=causal)
    vs = max(1.0, v.float().abs().max().item() / 4)
    d = (out[0].float().cpu() - ref[0].float()).abs()
    dl = (out[1].float().cpu() - ref[1].float()).abs()
    rowmax = d.amax(-1).flatten()
    worst = int(rowmax.argmax())
    print(f"{lib} case {i} {tuple(q.shape)} Sk={k.shape[2]} causal={causal}: |dO|/vs {d.max().item() / vs:.2e} "
          f"(worst row {worst} of {rowmax.numel()}, rows > 1e-2 vs: {int((rowmax > 1e-2 * vs).sum())}) "
          f"|dlse| {dl.max().item():.3g}", flush=True)
