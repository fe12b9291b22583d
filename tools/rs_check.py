"""Role-split int8 forward (P.V mode "rs") on the GPU: parity against the f16-mode kernel and the
oracle on small / grouped / ragged shapes, determinism, and config-3 kernel times against the other
modes (HIP events on the launch stream).  Dev tool:  python tools/rs_check.py [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import restate as R  # noqa: E402
from quantizedattention_amd import _lib  # noqa: E402
from quantizedattention_amd.attention_int8 import _int8_forward, _qk_scale  # noqa: E402


def run(q, k, v, pv):
    return _int8_forward(q, k, v, smooth=False, pv=pv)


def parity():
    g = torch.Generator().manual_seed(0)
    shapes = [((1, 2, 256, 128), 2), ((2, 3, 96, 128), 3), ((1, 4, 384, 128), 2), ((1, 2, 32, 128), 2),
              ((1, 8, 512, 128), 8)]
    for (B, H, S, D), Hkv in shapes:
        for Sk in (S, S + 64):
            q = torch.randn((B, H, S, D), generator=g).half()
            k = torch.randn((B, Hkv, Sk, D), generator=g).half()
            v = torch.randn((B, Hkv, Sk, D), generator=g).half()
            o_rs, l_rs = [t.float().cpu() for t in run(q.cuda(), k.cuda(), v.cuda(), "rs")[:2]]
            o_f, l_f = [t.float().cpu() for t in run(q.cuda(), k.cuda(), v.cuda(), "f16")[:2]]
            G = H // Hkv
            ref = R.int8_fwd(q, k.repeat_interleave(G, 1), v.repeat_interleave(G, 1))
            d_f = (o_rs - o_f).abs().max().item()
            d_ref = (o_rs - ref[0].float()).abs().max().item()
            d_lse = (l_rs - l_f).abs().max().item()
            print(f"shape {(B, H, S, D)} Hkv {Hkv} Sk {Sk}: |O_rs - O_f16| {d_f:.2e} |O_rs - O_oracle| "
                  f"{d_ref:.2e} |lse_rs - lse_f16| {d_lse:.2e}", flush=True)
            assert d_ref <= 1e-2, "rs vs oracle"


def timing(reps):
    B, H, S, D = 4, 32, 4096, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(3))
    outs = {}
    for pv in ("rs", "i8", "f16"):
        outs[pv] = run(q, k, v, pv)
    o1 = run(q, k, v, "rs")[0]
    print("rs deterministic:", torch.equal(o1, outs["rs"][0]), flush=True)
    print("config-3 |O_rs - O_i8|", (outs["rs"][0].float() - outs["i8"][0].float()).abs().max().item(),
          "|O_rs - O_f16|", (outs["rs"][0].float() - outs["f16"][0].float()).abs().max().item(), flush=True)
    # kernel-only times from the same quantised operands
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv = outs["rs"][:8]
    k_i8 = k_i8T.t()
    N = B * H * S
    st = _lib.stream_of(q)
    qks = float(torch.tensor(_qk_scale(D), dtype=torch.float32))
    P = _lib.ptr
    vop = torch.empty((N, D), dtype=torch.float16, device="cuda")
    vt = torch.empty((N, D), dtype=torch.int8, device="cuda")
    vdq = torch.empty((N, D), dtype=torch.float16, device="cuda")
    vi2 = torch.empty_like(v_i8)
    sv2 = torch.empty_like(sv)
    _lib.call("qattn_int8_quant_vop", P(v), P(vi2), P(sv2), P(vop), N, D, st)
    _lib.call("qattn_int8_quant_vt", P(v), P(vi2), P(sv2), P(vt), N, D, st)
    _lib.call("qattn_int8_quant", P(v), P(vi2), P(sv2), P(vdq), None, N, S, D, st)
    O2, lse2 = torch.empty_like(O), torch.empty_like(lse)
    fns = {
        "rs": lambda: _lib.call("qattn_int8_attn_fwd_rs", P(q_i8), P(sq), P(k_i8), P(sk), P(vop), P(O2),
                                P(lse2), B * H, S, S, 1, D, qks, st),
        "i8": lambda: _lib.call("qattn_int8_attn_fwd_i8pv_ex", P(q_i8), P(sq), P(k_i8), P(sk), P(vt), P(sv),
                                P(O2), P(lse2), B * H, S, S, 1, 0, D, qks, st),
        "f16": lambda: _lib.call("qattn_int8_attn_fwd_ex", P(q_i8), P(sq), P(k_i8), P(sk), P(vdq), P(O2),
                                 P(lse2), B * H, S, S, 1, 0, D, qks, st),
        "quant_vop": lambda: _lib.call("qattn_int8_quant_vop", P(v), P(vi2), P(sv2), P(vop), N, D, st),
        "quant_vt": lambda: _lib.call("qattn_int8_quant_vt", P(v), P(vi2), P(sv2), P(vt), N, D, st),
    }
    ops = 4 * B * H * S * S * D
    for rnd in range(2):
        line = []
        for name, fn in fns.items():
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            extra = f" ({ops / us / 1e6:.0f} TOP/s, {ops / us / 1e6 / 5033:.1%})" if "quant" not in name else ""
            line.append(f"{name} {us:.0f}us{extra}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    torch.cuda.init()
    parity()
    timing(int(sys.argv[1]) if len(sys.argv) > 1 else 10)
