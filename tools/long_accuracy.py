"""relL2 of the int8 forward against exact attention over long key ranges, for the library named by
QATTN_LIB (A/B dev tool for the KMAG re-bias period, csrc/int8_attn_fwd.hip `rebias`).

    QATTN_LIB=_ab/libqattn_<variant>.so python tools/long_accuracy.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd  # noqa: E402
from quantizedattention_amd.kv_cache import attention_int8_cached, quantize_kv  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(93)
out = []
for Sq, Sk, causal in ((256, 4096, False), (256, 65536, False), (64, 131072, True)):
    q = torch.randn((1, 2, Sq, 128), device="cuda", generator=g).half()
    k = torch.randn((1, 2, Sk, 128), device="cuda", generator=g).half()
    v = torch.randn((1, 2, Sk, 128), device="cuda", generator=g).half()
    if causal:
        O, _ = attention_int8_cached(q, quantize_kv(k, v), causal=True)
    else:
        O = helion_atten_int8_hl_dot_fwd(q, k, v)[0]
    s = (q.float() @ k.float().transpose(-1, -2)) / 128 ** 0.5
    if causal:
        mask = torch.arange(Sk, device="cuda")[None, :] > (Sk - Sq + torch.arange(Sq, device="cuda"))[:, None]
        s = s.masked_fill(mask, float("-inf"))
    ref = torch.softmax(s, dim=-1) @ v.float()
    out.append(f"Sk={Sk}{' causal' if causal else ''} relL2 {((O.float() - ref).norm() / ref.norm()).item():.4f}")
print(os.path.basename(os.environ.get("QATTN_LIB", "default")), " | ".join(out), flush=True)
