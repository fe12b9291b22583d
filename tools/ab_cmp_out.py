"""Bitwise diff of two O / lse dumps written by tools/ab_time.py (QATTN_AB_SAVE=<path>), e.g. the
in-tree build against an A/B variant (dev tool):  python tools/ab_cmp_out.py a.pt b.pt"""
import sys

import torch

a, b = (torch.load(p, weights_only=True) for p in sys.argv[1:3])
for k in ("O", "lse"):
    ne = a[k].view(torch.int16) != b[k].view(torch.int16)
    d = (a[k].float() - b[k].float()).abs()
    print(f"{k}: {int(ne.sum())} of {ne.numel()} differ, max abs {float(d.max()):.3g}")
    if k == "O" and ne.any():
        rows = ne.view(-1, a[k].shape[-1]).any(-1).nonzero().flatten()
        print(f"  {rows.numel()} rows differ; first {rows[:8].tolist()}")
