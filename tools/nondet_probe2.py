"""dq of the record backward against the recomputing backward (which it must equal bit for bit), over
repeated runs and workspace poison bytes (dev tool; run through tools/ab_run.sh to localise a
difference to a build option).

    python tools/nondet_probe2.py"""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward

name = os.path.basename(os.environ.get("QATTN_AB", "default"))


def probe(shape, causal, group=1, runs=6):
    B, H, S, D = shape
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    k, v = (torch.randn((B, H // group, S, D), device="cuda", generator=g).half() for _ in range(2))
    dO = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, q_bf, k_bf = _int8_forward(q, k, v, smooth=True, images=True,
                                                                         causal=causal)
    kw = dict(causal=causal, kv_heads=H // group, ws_chunk=0)
    ref = _int8_backward(dO, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf, k_bf, use_ws=False, **kw)
    out = []
    for i in range(runs):
        poison = (None, 0x00, 0x7F, 0x81)[i % 4]
        dq, dk, dv = _int8_backward(dO, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf, k_bf, use_ws=True,
                                    ws_poison=poison, **kw)
        torch.cuda.synchronize()
        d = (dq.view(torch.int16) != ref[0].view(torch.int16))
        rows = d.any(-1).nonzero()
        tiles = sorted({(int(r[0]), int(r[1]), int(r[2]) // 32, int(r[2]) % 32) for r in rows})
        out.append(f"poison={poison}: dq rows off {rows.shape[0]}"
                   f"{' e.g. (b,h,tile,row) ' + str(tiles[:3]) if tiles else ''}"
                   f" dk same {torch.equal(dk, ref[1])} dv same {torch.equal(dv, ref[2])}")
    print(f"{name} {shape} g{group} causal={causal}:", flush=True)
    for o in out:
        print("   ", o, flush=True)


R = int(os.environ.get("RUNS", "6"))
probe((2, 6, 3840, 64), False, runs=R)
probe((2, 6, 4096, 64), True, runs=R)
probe((2, 8, 1024, 64), True, group=4, runs=R)
if not os.environ.get("QUICK"):
    probe((2, 6, 3840, 128), False, runs=3)
