"""dK / dV of the fused dK+dV kernel against the separate dV and dK kernels (same P / dS
quantisation, so bit-identical), and the fused kernel's dS records of two runs (dev tool).

    python tools/nondet_probe3.py"""
import math, os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from quantizedattention_amd import _lib
from quantizedattention_amd.attention_int8 import _int8_forward, _qk_scale

name = os.path.basename(os.environ.get("QATTN_AB", "default"))


def rows_off(a, b, S):
    d = (a.view(torch.int16) != b.view(torch.int16)).reshape(-1, S, a.shape[-1]).any(-1)
    idx = d.nonzero()
    return f"{idx.shape[0]} rows off" + (f", e.g. (bh,row) {idx[:4].tolist()}" if idx.shape[0] else "")


def probe(shape):
    B, H, S, D = shape
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v, dO = (torch.randn((B, H, S, D), device="cuda", generator=g).half() for _ in range(4))
    O, lse, q_i8, k_i8T, v_i8, sq, sk, sv, _, q_bf, k_bf = _int8_forward(q, k, v, smooth=True, images=True)
    N = B * H * S
    dev = q.device
    st = _lib.stream_of(O)
    k_i8 = k_i8T.t().contiguous()
    dO_i8 = torch.empty((N, D), dtype=torch.int8, device=dev)
    sdO = torch.empty((N // 32,), dtype=torch.float16, device=dev)
    LD = torch.empty((N, 2), dtype=torch.float32, device=dev)
    dO_bf = torch.empty((N, D), dtype=torch.bfloat16, device=dev)
    lse16 = lse.to(torch.float16).contiguous()
    _lib.call("qattn_int8_bwd_prep", _lib.ptr(dO), _lib.ptr(O), _lib.ptr(lse16), _lib.ptr(dO_i8),
              _lib.ptr(sdO), _lib.ptr(LD), _lib.ptr(dO_bf), B * H, S, D, st)
    qks = float(torch.tensor(_qk_scale(D), dtype=torch.float32))
    sms = float(torch.tensor(1.0 / math.sqrt(D), dtype=torch.float32))
    sq, sk, sv = sq.contiguous(), sk.contiguous(), sv.contiguous()

    def run(fn, ws=None):
        dk = torch.full((B, H, S, D), float("nan"), dtype=torch.float16, device=dev)
        dv = torch.full((B, H, S, D), float("nan"), dtype=torch.float16, device=dev)
        args = [_lib.ptr(dO_i8), _lib.ptr(sdO), _lib.ptr(q_i8), _lib.ptr(sq), _lib.ptr(k_i8), _lib.ptr(sk),
                _lib.ptr(v_i8), _lib.ptr(sv), _lib.ptr(LD), _lib.ptr(q_bf), _lib.ptr(dO_bf), _lib.ptr(dk),
                _lib.ptr(dv)]
        if ws is not None:
            args.append(_lib.ptr(ws))
        _lib.call(fn, *args, B * H, S, D, qks, sms, st)
        torch.cuda.synchronize()
        return dk, dv

    dk_f, dv_f = run("qattn_int8_bwd_dkdv")
    _, dv_s = run("qattn_int8_bwd_dv")
    dk_s, _ = run("qattn_int8_bwd_dk")
    print(f"{name} {shape}: fused vs separate: dk {rows_off(dk_f, dk_s, S)}; dv {rows_off(dv_f, dv_s, S)}",
          flush=True)
    nb = _lib.load().qattn_int8_bwd_ws_bytes(B * H, S, S)
    recs = []
    for fill in (0x00, 0x7F):
        ws = torch.full((nb,), fill, dtype=torch.uint8, device=dev)
        dk_w, dv_w = run("qattn_int8_bwd_dkdv_ws", ws)
        recs.append(ws)
        print(f"   records run (fill {fill:#x}): dk vs fused {rows_off(dk_w, dk_f, S)}; dv {rows_off(dv_w, dv_f, S)}",
              flush=True)
    nt = S // 32
    r8 = [w[: B * H * nt * nt * 1024].view(B * H, nt, nt, 64, 16) for w in recs]   # [bh, qt, kt, lane, byte]
    diff = (r8[0] != r8[1])
    bad = diff.any(-1).any(-1)                                                      # [bh, qt, kt]
    idx = bad.nonzero()
    print(f"   records differing between runs: {idx.shape[0]} of {bad.numel()}"
          + (f"; (bh,qt,kt) e.g. {idx[:6].tolist()}; bytes per record lane differing: "
             f"{diff[tuple(idx[0])].any(0).nonzero().flatten().tolist()}" if idx.shape[0] else ""), flush=True)


probe((2, 6, 3840, 64))
probe((2, 6, 1024, 64))
probe((1, 4, 3840, 128))
