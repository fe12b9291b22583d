"""Time the JVP forward at config 5 (bf16 inputs) for the library named by QATTN_LIB (A/B dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
x = [torch.randn((2, 16, 2048, 128), device="cuda", generator=g).bfloat16() for _ in range(6)]
t = bench.event_time(lambda: helion_attention_jvp_forward_fp32(*x), 10)
print(os.environ.get("QATTN_LIB", "default"), "jvp cfg5 ms", round(t, 4), flush=True)
