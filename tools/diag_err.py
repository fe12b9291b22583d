"""Locate the int8 forward's largest deviations from the oracle (debugging aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import restate as R  # noqa: E402
from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd  # noqa: E402

shape = tuple(int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,2,512,128").split(","))
g = torch.Generator().manual_seed(1)
q, k, v = (torch.randn(shape, generator=g).half() for _ in range(3))
ref = R.int8_fwd(q, k, v)
out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda())
torch.cuda.synchronize()
B, H, S, D = shape
e = (out[0].float().cpu() - ref[0].float()).abs().reshape(B * H, S, D)
rowerr = e.amax(-1)
idx = torch.nonzero(rowerr > 0.004)
print("rows with err > 4e-3:", idx.shape[0], "of", B * H * S)
for bh, r in idx[:40].tolist():
    d = int(e[bh, r].argmax())
    print(f"bh {bh} row {r} (row%32 {r % 32}, q-tile {r // 128}, wave {(r % 128) // 32}) d {d} "
          f"err {rowerr[bh, r]:.4f} got {out[0].reshape(B*H,S,D)[bh, r, d].item():.4f} "
          f"ref {ref[0].reshape(B*H,S,D)[bh, r, d].item():.4f} lse {out[1].reshape(B*H,S)[bh, r].item():.3f}/"
          f"{ref[1].reshape(B*H,S)[bh, r].item():.3f}")
hist = torch.histc(rowerr, bins=10, min=0, max=0.015)
print("row err histogram (0..0.015):", hist.tolist())
