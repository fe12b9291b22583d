"""Repeat the int8 backward on one GQA causal case and count runs whose dq / dk / dv differ from the
first (a race shows up as run-to-run differences; dev tool).   python tools/race_check.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.attention_int8 import _int8_backward, helion_atten_int8_hl_dot_fwd  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for (B, Hq, Hkv, S, D, causal) in [(2, 6, 3, 256, 64, True), (2, 4, 4, 512, 128, True),
                                   (1, 8, 2, 1024, 128, True), (2, 6, 3, 256, 64, False)]:
    g = torch.Generator(device="cuda").manual_seed(12)
    q = torch.randn((B, Hq, S, D), device="cuda", generator=g).half() * 2
    k = torch.randn((B, Hkv, S, D), device="cuda", generator=g).half() * 2
    v = torch.randn((B, Hkv, S, D), device="cuda", generator=g).half()
    dO = torch.randn((B, Hq, S, D), device="cuda", generator=g).half()
    O, lse, qi, kiT, vi, sq, sk, sv, _, _ = helion_atten_int8_hl_dot_fwd(q, k, v, causal=causal)
    ref = None
    bad = {"dq": 0, "dk": 0, "dv": 0}
    for r in range(reps):
        out = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, causal=causal, kv_heads=Hkv, use_ws=True)
        torch.cuda.synchronize()
        if ref is None:
            ref = [t.clone() for t in out]
            rec = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, causal=causal, kv_heads=Hkv, use_ws=False)
            same = [torch.equal(a, b) for a, b in zip(ref, rec)]
            print("ws vs recompute bit-identical:", same, flush=True)
            continue
        for n, a, b in zip(("dq", "dk", "dv"), out, ref):
            bad[n] += int(not torch.equal(a, b))
    print((B, Hq, Hkv, S, D, causal), "runs differing from the first:", bad, flush=True)
