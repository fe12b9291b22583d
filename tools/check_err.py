"""Print the int8 forward's max |O - O_oracle| and lse error over a few shapes (margin tracking)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import restate as R  # noqa: E402
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd  # noqa: E402

for shape in [(1, 2, 128, 64), (1, 2, 256, 128), (2, 2, 512, 128), (1, 4, 1024, 128), (1, 2, 1024, 64)]:
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.randn(shape, generator=g).half() for _ in range(3))
    ref = R.int8_fwd(q, k, v)
    out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda())
    torch.cuda.synchronize()
    e = (out[0].float().cpu() - ref[0].float()).abs()
    le = (out[1].float().cpu() - ref[1].float()).abs().max().item()
    print(f"{shape}: max|dO| {e.max().item():.5f}  mean {e.mean().item():.2e}  lse {le:.4f}", flush=True)
