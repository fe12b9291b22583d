"""Time the int8 backward kernels (dV, dK, dQ) of the library named by QATTN_LIB (A/B dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

B, H, S, D = 4, 32, 4096, 128
g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
kt = bench.int8_kernel_times(q, k, v, dO, 10)
print(os.environ.get("QATTN_LIB", "default"),
      {k_: round(v_ * 1e3, 1) for k_, v_ in kt.items() if "bwd" in k_ or "fwd" in k_}, flush=True)
