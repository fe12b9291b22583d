"""The role-split int8 forward (qattn_int8_attn_fwd_rs_ex, csrc/int8_attn_fwd.hip): the same
computation as qattn_int8_attn_fwd_i8pv_ex, checked against the oracle (O <= 1e-2, lse within 2 fp16
ulp) and against the single-role kernel on the same operands."""
import math

import pytest
import torch

from quantizedattention_amd import _lib

pytestmark = pytest.mark.gpu


def _operands(q, k, v):
    from quantizedattention_amd.attention_int8 import _qk_scale
    B, H, S, D = q.shape
    Hkv, Sk = k.shape[1], k.shape[2]
    N, Nkv = B * H * S, B * Hkv * Sk
    dev = q.device
    st = _lib.stream_of(q)
    e = lambda *s, dt: torch.empty(s, dtype=dt, device=dev)  # noqa: E731
    qi, ki, vi, vt = e(N, D, dt=torch.int8), e(Nkv, D, dt=torch.int8), e(Nkv, D, dt=torch.int8), e(Nkv, D, dt=torch.int8)
    sq, sk, sv = e(N // 32, dt=torch.float16), e(Nkv // 32, dt=torch.float16), e(Nkv // 32, dt=torch.float16)
    P = _lib.ptr
    _lib.call("qattn_int8_quant", P(q), P(qi), P(sq), None, None, N, S, D, st)
    _lib.call("qattn_int8_quant", P(k), P(ki), P(sk), None, None, Nkv, Sk, D, st)
    _lib.call("qattn_int8_quant_vt", P(v), P(vi), P(sv), P(vt), Nkv, D, st)
    qks = float(torch.tensor(_qk_scale(D), dtype=torch.float32))
    return (qi, sq, ki, sk, vt, sv), (B * H, S, Sk, H // Hkv, 0, D, qks, st)


def _run(entry, ops, shape, O_shape, dev):
    O = torch.empty(O_shape, dtype=torch.float16, device=dev)
    lse = torch.empty(O.numel() // O_shape[-1], dtype=torch.float16, device=dev)
    _lib.call(entry, *(_lib.ptr(t) for t in ops), _lib.ptr(O), _lib.ptr(lse), *shape)
    return O, lse


@pytest.mark.parametrize("shape", [(1, 2, 256, 128, 2, 256), (2, 4, 160, 128, 2, 512), (1, 4, 4096, 128, 4, 4096)])
def test_rs_forward_matches_oracle_and_single_role(lib, shape):
    from oracle import restate as R
    B, H, S, D, Hkv, Sk = shape
    g = torch.Generator(device="cuda").manual_seed(21)
    q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    k = torch.randn((B, Hkv, Sk, D), device="cuda", generator=g).half()
    v = torch.randn((B, Hkv, Sk, D), device="cuda", generator=g).half()
    ops, shp = _operands(q, k, v)
    Ors, lrs = _run("qattn_int8_attn_fwd_rs_ex", ops, shp, q.shape, q.device)
    Oi8, li8 = _run("qattn_int8_attn_fwd_i8pv_ex", ops, shp, q.shape, q.device)
    assert torch.isfinite(Ors).all()
    # same operands, same recipe: only the bias constant of the accumulators differs
    assert (Ors.float() - Oi8.float()).abs().max().item() <= 2e-3
    assert (lrs.float() - li8.float()).abs().max().item() <= 2e-2
    nh = 1 if S >= 4096 else B * H   # full-size: one head against the oracle
    G = H // Hkv
    for bh in range(nh):
        b, hh = divmod(bh, H)
        ref = R.int8_fwd(q[b:b + 1, hh:hh + 1].cpu(), k[b:b + 1, hh // G:hh // G + 1].cpu(),
                         v[b:b + 1, hh // G:hh // G + 1].cpu())
        err = (Ors[b, hh].float().cpu() - ref[0][0, 0].float()).abs().max().item()
        assert err <= 1e-2, (bh, err)
        lerr = (lrs.view(B, H, S)[b, hh].float().cpu() - ref[1].float().view(S)).abs()
        assert (lerr <= 2 * 2.0 ** -10 * ref[1].float().abs().view(S).clamp_min(1) + 1e-3).all()


def test_rs_forward_rejects_unsupported(lib):
    f = _lib.load().qattn_int8_attn_fwd_rs_ex
    assert f(*([None] * 5), _lib.ptr(torch.empty(1)), None, None, 4, 64, 64, 1, 1, 128, 0.1, None) == 1   # causal
    assert f(*([None] * 5), _lib.ptr(torch.empty(1)), None, None, 4, 64, 64, 1, 0, 64, 0.1, None) == 1    # D = 64
