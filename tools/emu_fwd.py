"""Debug aid: a CPU emulation of the int8 forward kernel's own algorithm (per-tile deferred max per
32-row wave, f16 S / d / e, trunc(127 e), f16 operands), compared element-wise with the GPU."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import restate as R  # noqa: E402


def emulate(q, k, v, thr=8.0):
    B, H, S, D = q.shape
    BH = B * H
    qks = R.qk_scale(D)
    qi, sq = R.quant_blocks(q.reshape(BH, S, D))
    ki, sk = R.quant_blocks(k.reshape(BH, S, D))
    vi, sv = R.quant_blocks(v.reshape(BH, S, D))
    vdq = (vi.float() * sv.float().repeat_interleave(32, 1)[..., None]).half().double()
    O = torch.zeros(BH, S, D, dtype=torch.float64)
    l = torch.zeros(BH, S, 1, dtype=torch.float64)
    m = torch.full((BH, S, 1), float("-inf"))
    cq = (sq.float() * qks).repeat_interleave(32, 1)[..., None]
    for t in range(S // 32):
        ks = slice(32 * t, 32 * t + 32)
        acc = (qi.double() @ ki[:, ks].double().transpose(1, 2))
        c = (cq * sk[:, t].float()[:, None, None]).double()
        S16 = (acc * c).half()
        rm = S16.amax(-1, keepdim=True).float()
        g = (rm.reshape(BH, S // 32, 32) > (m.reshape(BH, S // 32, 32) + thr)).any(-1, keepdim=True)
        g = g.expand(-1, -1, 32).reshape(BH, S, 1)
        nm = torch.where(g, torch.maximum(m, rm), m)
        r = torch.where(g, torch.exp2((m - nm).half().float()), torch.ones_like(m))
        m = nm
        l = l * r.double()
        O = O * r.double()
        er = torch.exp2((rm - m).half().float())
        sp = (er / 127).half()
        d = (S16.float() - rm).half()
        e = torch.exp2(d.float()).half()
        Pi = torch.trunc(e.double() * 127)
        w = (Pi * sp.double()).half()
        l = l + e.double().sum(-1, keepdim=True) * er.double()
        O = O + w.double() @ vdq[:, ks]
    return (O / l).half().view(B, H, S, D)


if __name__ == "__main__":
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    shape = tuple(int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,2,512,128").split(","))
    g = torch.Generator().manual_seed(1)
    q, k, v = (torch.randn(shape, generator=g).half() for _ in range(3))
    em = emulate(q, k, v)
    ref = R.int8_fwd(q, k, v)[0]
    out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda())[0].cpu()
    B, H, S, D = shape
    print("emu vs oracle", (em.float() - ref.float()).abs().max().item())
    dif = (out.float() - em.float()).abs().reshape(B * H, S, D)
    print("gpu vs emu max", dif.max().item(), "mean", dif.mean().item())
    rowd = dif.amax(-1)
    bad = torch.nonzero(rowd > 2e-3)
    print("rows gpu-emu > 2e-3:", bad.shape[0])
    for bh, r in bad[:20].tolist():
        print(f"  bh {bh} row {r} q-tile {r // 128} wave {(r % 128) // 32} lane-row {r % 32} "
              f"diff {rowd[bh, r]:.4f}")
