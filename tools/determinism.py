"""Run the int8 forward repeatedly on the same inputs; report bitwise run-to-run differences."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd  # noqa: E402

shape = tuple(int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,2,512,128").split(","))
g = torch.Generator().manual_seed(1)
q, k, v = (torch.randn(shape, generator=g).half().cuda() for _ in range(3))
base = helion_atten_int8_hl_dot_fwd(q, k, v)[0].clone()
ndiff = []
for i in range(10):
    o = helion_atten_int8_hl_dot_fwd(q, k, v)[0]
    ndiff.append(((o != base).sum().item(), (o.float() - base.float()).abs().max().item()))
print("run-to-run (n differing, max diff):", ndiff, flush=True)
