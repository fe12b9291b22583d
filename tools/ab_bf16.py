"""Time the bf16 forward / backward kernels of the library named by QATTN_LIB (A/B dev tool).

    python tools/ab_bf16.py [B,H,S,D] [causal] [f = forward only]
"""
import hashlib
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd.attention_bf16 import (  # noqa: E402
    helion_atten_bf16_fwd_training, helion_flash_atten_2_algo_4_bwd)

B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,32,4096,128").split(","))
causal = len(sys.argv) > 2 and sys.argv[2] == "1"
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
k = torch.randn((B, H, S, D), device="cuda", generator=g).half()
v = torch.randn((B, H, S, D), device="cuda", generator=g).bfloat16()
dO = torch.randn((B, H, S, D), device="cuda", generator=g)
O, lse = helion_atten_bf16_fwd_training(q, k, v, causal)


def timed(f, n=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


tf = timed(lambda: helion_atten_bf16_fwd_training(q, k, v, causal))
fwd_only = len(sys.argv) > 3 and sys.argv[3] == "f"
tb = 1.0 if fwd_only else timed(lambda: helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, causal, dO))
flop = 4 * B * H * S * S * D
peak = 256 * 4096 * 2.4e9
O, lse = helion_atten_bf16_fwd_training(q, k, v, causal)
digest = hashlib.sha256(O.cpu().numpy().tobytes() + lse.cpu().numpy().tobytes()).hexdigest()[:12]
print(f"{os.environ.get('QATTN_LIB', 'default')}: O/lse {digest}  fwd {tf * 1e3:.1f} us "
      f"({flop / tf / 1e9:.0f} TFLOP/s, {flop / tf / 1e-3 / peak * 100:.1f}% bf16 peak)  "
      f"bwd {tb * 1e3:.1f} us ({2.5 * flop / tb / 1e9:.0f} TFLOP/s)", flush=True)
