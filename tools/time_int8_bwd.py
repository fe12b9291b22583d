"""Time the int8 backward call (dS-record path) at config 3, non-causal and causal (dev tool)."""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward
B, H, S, D = 4, 32, 4096, 128
for causal in (False, True):
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
    dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, q_bf, k_bf = _int8_forward(q, k, v, smooth=True, images=True, causal=causal)
    ts = []
    for i in range(10):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); _int8_backward(dO, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf, k_bf, causal=causal); b.record()
        torch.cuda.synchronize()
        if i >= 2: ts.append(a.elapsed_time(b))
    print("causal", causal, "bwd ms", round(sorted(ts)[len(ts)//2], 3), flush=True)
