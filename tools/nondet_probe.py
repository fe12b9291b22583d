"""Run-to-run differences of the int8 forward and record backward at D = 64 (dev tool): per tensor,
how many elements differ between two runs on the same inputs, and where.

    python tools/nondet_probe.py"""
import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward


def where(a, b):
    d = (a.view(torch.int16) != b.view(torch.int16)) if a.dtype == torch.float16 else (a != b)
    n = int(d.sum())
    if n == 0:
        return "same"
    idx = d.nonzero()
    rows = idx[:, :-1].unique(dim=0)
    return (f"{n} differ, max|diff| {float((a.float() - b.float()).abs().max()):.3g}, rows {rows.shape[0]}, "
            f"first {idx[0].tolist()} last {idx[-1].tolist()}")


def probe(shape, causal, group=1, use_ws=True):
    B, H, S, D = shape
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    k, v = (torch.randn((B, H // group, S, D), device="cuda", generator=g).half() for _ in range(2))
    dO = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    runs = []
    for _ in range(2):
        f = _int8_forward(q, k, v, smooth=True, images=True, causal=causal)
        O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, q_bf, k_bf = f
        grads = _int8_backward(dO, q_i8, sq, k_i8T, sk, v_i8, sv, O, lse, q_bf, k_bf, causal=causal,
                               kv_heads=H // group, use_ws=use_ws, ws_chunk=0)
        torch.cuda.synchronize()
        runs.append((O, lse, q_i8, v_i8) + tuple(grads))
    names = ("O", "lse", "q_i8", "v_i8", "dq", "dk", "dv")
    print(f"{shape} g{group} causal={causal} ws={use_ws}:", flush=True)
    for n, a, b in zip(names, *runs):
        print(f"  {n}: {where(a, b)}", flush=True)


probe((2, 6, 3840, 64), True)
probe((2, 6, 3840, 64), True, use_ws=False)
probe((2, 6, 3840, 64), False)
probe((2, 6, 4096, 64), True)
probe((2, 8, 1024, 64), True, group=4)
probe((2, 8, 1024, 128), True, group=4)
probe((2, 8, 1056, 128), True)
