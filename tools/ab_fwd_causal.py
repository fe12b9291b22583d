"""Time the int8 forward call (quantisers + attention) at config 3, causal and not (dev A/B tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from quantizedattention_amd.attention_int8 import _int8_forward  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
q, k, v = (torch.randn((4, 32, 4096, 128), device="cuda", generator=g).half() for _ in range(3))
r = {c: round(bench.event_time(lambda: _int8_forward(q, k, v, smooth=True, causal=c), 10), 4)
     for c in (False, True)}
print(os.environ.get("QATTN_LIB", "default"), "fwd ms (non-causal, causal)", r, flush=True)
