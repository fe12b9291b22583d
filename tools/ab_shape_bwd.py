"""int8 kernel times at two shapes of equal B·H·S² (per-workgroup fixed cost probe, dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

for B, H, S in ((4, 32, 4096), (4, 128, 2048), (4, 8, 8192)):
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((B, H, S, 128), device="cuda", generator=g).half() for _ in range(3))
    dO = (torch.randn((B, H, S, 128), device="cuda", generator=g) * 1e-3).half()
    kt = bench.int8_kernel_times(q, k, v, dO, 6)
    keep = ("int8_attn_fwd_kernel", "int8_bwd_dkdv_kernel<dK+dV, dS out>", "int8_bwd_dqw_kernel")
    print((B, H, S), {k_: round(v_ * 1e3, 1) for k_, v_ in kt.items() if k_ in keep}, flush=True)
    del q, k, v, dO
