"""Time the bf16 backward at config 3: dS records (default), fused dK+dV, split dV/dK (dev A/B).

    python3 tools/ab_bf16_bwd.py [B,H,S,D] [causal]
Prints the median event time of each backward call; also usable under rocprofv3 --kernel-trace.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd import attention_bf16 as A  # noqa: E402

B, H, S, D = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,32,4096,128").split(","))
causal = len(sys.argv) > 2 and sys.argv[2] == "1"
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
k = torch.randn((B, H, S, D), device="cuda", generator=g).half()
v = torch.randn((B, H, S, D), device="cuda", generator=g).bfloat16()
dO = torch.randn((B, H, S, D), device="cuda", generator=g)
O, lse = A.helion_atten_bf16_fwd_training(q, k, v, causal)
res, hs = {}, {}
ENTRIES = os.environ.get("QATTN_AB_ENTRIES", "auto,ws,qattn_bf16_bwd_ex,qattn_bf16_bwd_split_ex").split(",")
for entry in ENTRIES:
    A._BWD_ENTRY = entry
    ts = []
    for i in range(8):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = A.helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, causal, dO)
        b.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(a.elapsed_time(b))
    res[entry] = sorted(ts)[len(ts) // 2]
    # checksum of the gradient bits (on the GPU: bit-identical outputs give equal sums)
    hs[entry] = sum(int(t.float().view(torch.int32).to(torch.int64).sum()) * (i + 1) for i, t in enumerate(out[:3]))
print(os.environ.get("QATTN_LIB", "default"), {k: round(v, 3) for k, v in res.items()}, hs)
