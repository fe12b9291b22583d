"""Dump the dS-record workspace of one record backward (dev tool: compare two library builds).
    QATTN_LIB=<lib> python tools/ws_records.py <out.pt> [B,H,S,D]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import quantizedattention_amd.attention_int8 as A  # noqa: E402
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd  # noqa: E402

B, H, S, D = (int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,128,64").split(","))
g = torch.Generator().manual_seed(31)
q, k, v = (torch.randn((B, H, S, D), generator=g).half().cuda() for _ in range(3))
dO = torch.randn((B, H, S, D), generator=torch.Generator().manual_seed(32)).half().cuda()
O, lse, qi, kiT, vi, sq, sk, sv, _, _ = helion_atten_int8_hl_dot_fwd(q, k, v)
orig, cap = torch.empty, {}


def spy(*a, **kw):
    t = orig(*a, **kw)
    if kw.get("dtype") == torch.uint8 and len(a) == 1:
        t.fill_(0x55)
        cap["ws"] = t
    return t


A.torch.empty = spy
dq, dk, dv = A._int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, use_ws=True)
A.torch.empty = orig
torch.cuda.synchronize()
torch.save({"ws": cap["ws"].cpu(), "dq": dq.cpu(), "dk": dk.cpu(), "dv": dv.cpu()}, sys.argv[1])
print("saved", sys.argv[1])
