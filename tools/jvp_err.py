"""Error of the fp32-mode JVP kernel vs torch.func.jvp of the baseline in float64 (dev tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import restate as R  # noqa: E402
from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32  # noqa: E402

for shape in [(1, 2, 128, 64), (2, 2, 256, 128), (1, 2, 1024, 128)]:
    g = torch.Generator().manual_seed(11)
    ins = [torch.randn(shape, generator=g) for _ in range(6)]
    O, tO, lse = helion_attention_jvp_forward_fp32(*(t.cuda() for t in ins))
    f = lambda a, b, c: R.baseline_pytorch_attention(a, b, c, None, False)
    f64 = lambda a, b, c: torch.softmax(a @ b.transpose(2, 3) / a.shape[-1] ** 0.5, dim=-1) @ c
    Od, tOd = torch.func.jvp(f64, tuple(t.double() for t in ins[:3]), tuple(t.double() for t in ins[3:]))
    Of, tOf = torch.func.jvp(f, tuple(ins[:3]), tuple(ins[3:]))
    print(shape, "kernel vs f64: O %.2e tO %.2e | cpu-f32 vs f64: O %.2e tO %.2e | max|tO| %.2f" % (
        (O.cpu().double() - Od).abs().max(), (tO.cpu().double() - tOd).abs().max(),
        (Of.double() - Od).abs().max(), (tOf.double() - tOd).abs().max(), tOd.abs().max()), flush=True)
