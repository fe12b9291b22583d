"""bf16 path on the GPU vs the CPU restatement (oracle/restate.py).

Tolerances: forward O max-abs <= 5e-3 vs the restatement at the same k-tile (16),
lse max-abs <= 5e-3; gradients relL2 <= 1e-2 vs the corrected restatement (fp32) and <= 2e-2 vs
fp32 autograd of baseline_pytorch_attention (non-causal).
"""
import pytest
import torch

from oracle import restate as R

pytestmark = pytest.mark.gpu

SHAPES = [(1, 2, 128, 64), (1, 2, 256, 128), (2, 3, 96, 128), (1, 1, 64, 64), (1, 4, 512, 128)]


def _inputs(shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    q, k, v = [torch.randn(shape, generator=g) for _ in range(3)]
    return q.half(), k.half(), v.bfloat16()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("causal", [False, True])
def test_bf16_fwd_matches_oracle(lib, shape, causal):
    from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training
    q, k, v = _inputs(shape)
    O_ref, lse_ref = R.bf16_fwd(q, k, v, causal, kt=16)
    O, lse = helion_atten_bf16_fwd_training(q.cuda(), k.cuda(), v.cuda(), causal)
    torch.cuda.synchronize()
    assert O.dtype == torch.float32 and lse.shape == (shape[0] * shape[1], shape[2])
    err = (O.cpu() - O_ref).abs().max().item()
    assert err <= 5e-3, err
    lerr = (lse.cpu() - lse_ref).abs().max().item()
    assert lerr <= 5e-3, lerr


def test_bf16_fwd_beta_rule_forced(lib):
    """Rows with several near-equal maxima force the doubling branch (rule 26: test the rare path)."""
    from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training
    B, H, S, D = 1, 2, 128, 64
    q, k, v = _inputs((B, H, S, D), seed=5)
    k[:, :, 16:20] = q[:, :, 0:1].expand(-1, -1, 4, -1) * 2   # duplicated maxima for row 0
    k[:, :, 40:48] = k[:, :, 40:41]                           # identical keys -> ties everywhere
    O_ref, lse_ref = R.bf16_fwd(q, k, v, False, kt=16)
    O, lse = helion_atten_bf16_fwd_training(q.cuda(), k.cuda(), v.cuda(), False)
    assert (O.cpu() - O_ref).abs().max().item() <= 5e-3
    assert (lse.cpu() - lse_ref).abs().max().item() <= 5e-3


@pytest.mark.parametrize("shape", [(1, 2, 128, 64), (1, 2, 256, 128), (2, 2, 192, 128), (1, 4, 512, 128)])
@pytest.mark.parametrize("causal", [False, True])
def test_bf16_bwd_matches_oracle(lib, shape, causal):
    from quantizedattention_amd.attention_bf16 import (helion_atten_bf16_fwd_training,
                                                       helion_flash_atten_2_algo_4_bwd)
    q, k, v = _inputs(shape, seed=11)
    dO = torch.randn(shape, generator=torch.Generator().manual_seed(12))
    O, lse = helion_atten_bf16_fwd_training(q.cuda(), k.cuda(), v.cuda(), causal)
    dq, dk, dv = helion_flash_atten_2_algo_4_bwd(q.cuda(), k.cuda(), v.cuda(), O, lse, causal,
                                                 dO.cuda())
    torch.cuda.synchronize()
    rq, rk, rv = R.bf16_bwd(q, k, v, O.cpu(), lse.cpu(), causal, dO)
    for name, a, b in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        assert a.dtype == torch.float32
        assert _rel(a.cpu(), b) <= 1e-2, (name, _rel(a.cpu(), b))
    if not causal:
        tq, tk, tv = R.attention_grads_truth(q, k, v, dO, False)
        for name, a, b in (("dq", dq, tq), ("dk", dk, tk), ("dv", dv, tv)):
            assert _rel(a.cpu(), b) <= 2e-2, (name, _rel(a.cpu(), b))


def test_bf16_autograd_end_to_end(lib):
    """flash_atten_2_bf16 through torch.autograd: grads land on fp16/fp16/bf16 leaves (bf16:85)."""
    from quantizedattention_amd.attention_bf16 import flash_atten_2_bf16
    shape = (1, 2, 256, 64)
    q, k, v = _inputs(shape, seed=21)
    qd, kd, vd = (t.cuda().requires_grad_(True) for t in (q, k, v))
    out = flash_atten_2_bf16(qd, kd, vd, causal=False)
    gt = torch.randn(shape, generator=torch.Generator().manual_seed(22)).cuda()
    torch.nn.functional.mse_loss(out, gt).backward()
    assert qd.grad.dtype == torch.float16 and vd.grad.dtype == torch.bfloat16
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = R.baseline_pytorch_attention(qf, kf, vf, 64, False)
    torch.nn.functional.mse_loss(ref, gt.cpu()).backward()
    for a, b in ((qd.grad, qf.grad), (kd.grad, kf.grad), (vd.grad, vf.grad)):
        assert _rel(a.float().cpu(), b) <= 3e-2


@pytest.mark.parametrize("hq,hkv,sq,sk,causal", [(4, 2, 128, 128, False), (4, 1, 96, 192, True),
                                                 (6, 2, 128, 64, True)])
def test_bf16_gqa_fwd_bwd(lib, hq, hkv, sq, sk, causal):
    """Grouped-query attention (SURVEY §8f N2 extension) vs the oracle on expanded heads: same
    tolerances as the square tests; dk, dv sum over each group of query heads."""
    from quantizedattention_amd.attention_bf16 import (helion_atten_bf16_fwd_training,
                                                       helion_flash_atten_2_algo_4_bwd)
    g = torch.Generator().manual_seed(31)
    D = 64
    q = torch.randn((1, hq, sq, D), generator=g).half()
    k = torch.randn((1, hkv, sk, D), generator=g).half()
    v = torch.randn((1, hkv, sk, D), generator=g).bfloat16()
    dO = torch.randn((1, hq, sq, D), generator=g)
    O, lse = helion_atten_bf16_fwd_training(q.cuda(), k.cuda(), v.cuda(), causal)
    O_ref, lse_ref = R.bf16_fwd(q, k, v, causal, kt=16)
    assert (O.cpu() - O_ref).abs().max().item() <= 5e-3
    assert (lse.cpu() - lse_ref).abs().max().item() <= 5e-3
    dq, dk, dv = helion_flash_atten_2_algo_4_bwd(q.cuda(), k.cuda(), v.cuda(), O, lse, causal, dO.cuda())
    torch.cuda.synchronize()
    rq, rk, rv = R.bf16_bwd(q, k, v, O.cpu(), lse.cpu(), causal, dO)
    assert dk.shape == k.shape and dv.shape == v.shape and dq.shape == q.shape
    for name, a, b in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        assert _rel(a.cpu(), b) <= 1e-2, (name, _rel(a.cpu(), b))


@pytest.mark.parametrize("hq,hkv,sq,sk,d", [(4, 4, 1024, 1024, 128), (4, 2, 512, 1024, 64),
                                          (2, 1, 384, 256, 128), (2, 2, 1056, 1056, 64)])
def test_bf16_fwd_causal_vsuffix_matches_tile_loop(lib, hq, hkv, sq, sk, d):
    """The causal V-suffix path (qattn_bf16_fwd_ws_ex) against the full masked tile loop
    (qattn_bf16_fwd_ex, no workspace): the masked sub-tiles' constant P times the suffix sum of V
    equals their P.V MFMAs up to fp32 summation order; GQA, Sq != Sk, ragged workgroups
    (1056 = 8 x 128 + 32).  The tile loop adds 16 p per sub-tile to l (and p.V to O) one sub-tile at
    a time, as the reference does (bf16:279-285), and those fp32 additions of a small term to a larger
    one round the same way each time: measured 2.2e-5 on O and 1.0e-5 on lse at 1024 keys, in the
    first rows (the longest masked suffix), falling off with the row.  Bound: 1e-4 (the oracle
    tolerance is 5e-3)."""
    import math
    from quantizedattention_amd import _lib
    g = torch.Generator().manual_seed(41)
    q = torch.randn((1, hq, sq, d), generator=g).half().cuda()
    k = torch.randn((1, hkv, sk, d), generator=g).half().cuda()
    v = torch.randn((1, hkv, sk, d), generator=g).bfloat16().cuda()
    qks = float(torch.tensor(1.0 / math.sqrt(d) * 1.44269504, dtype=torch.float32))
    outs = []
    for use_ws in (False, True):
        O = torch.full((hq, sq, d), float("nan"), device="cuda")
        lse = torch.full((hq, sq), float("nan"), device="cuda")
        ws = torch.full((lib.qattn_bf16_fwd_ws_bytes(hkv, sk, d) // 4,), float("nan"), device="cuda")
        fn = "qattn_bf16_fwd_ws_ex" if use_ws else "qattn_bf16_fwd_ex"
        args = (_lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(O), _lib.ptr(lse), hq, sq, sk, hq // hkv,
                1, d, qks) + ((_lib.ptr(ws),) if use_ws else ()) + (_lib.stream_of(q),)
        _lib.call(fn, *args)
        outs.append((O, lse))
    torch.cuda.synchronize()
    (O0, l0), (O1, l1) = outs
    assert torch.isfinite(O1).all() and torch.isfinite(l1).all()
    assert (O1 - O0).abs().max().item() <= 1e-4
    assert (l1 - l0).abs().max().item() <= 1e-4


def test_bf16_fwd_causal_vsuffix_config2(lib):
    """Config 2 (4,32,2048,128), causal: the V-suffix forward against the full masked tile loop.
    The last 32-query block of each head has no masked suffix, so its rows are bit-identical; the
    rest differ only by the tile loop's fp32 drift (see the test above): |dO|, |dlse| <= 5e-4."""
    import math
    from quantizedattention_amd import _lib
    B, H, S, D = 4, 32, 2048, 128
    g = torch.Generator(device="cuda").manual_seed(2)
    q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    k = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    v = torch.randn((B, H, S, D), device="cuda", generator=g).bfloat16()
    qks = float(torch.tensor(1.0 / math.sqrt(D) * 1.44269504, dtype=torch.float32))
    ws = torch.empty(lib.qattn_bf16_fwd_ws_bytes(B * H, S, D) // 4, device="cuda")
    outs = []
    for use_ws in (False, True):
        O = torch.empty((B * H, S, D), device="cuda")
        lse = torch.empty((B * H, S), device="cuda")
        args = (_lib.ptr(q), _lib.ptr(k), _lib.ptr(v), _lib.ptr(O), _lib.ptr(lse), B * H, S, S, 1, 1, D,
                qks) + ((_lib.ptr(ws),) if use_ws else ()) + (_lib.stream_of(q),)
        _lib.call("qattn_bf16_fwd_ws_ex" if use_ws else "qattn_bf16_fwd_ex", *args)
        outs.append((O, lse))
    torch.cuda.synchronize()
    (O0, l0), (O1, l1) = outs
    assert torch.equal(O1[:, S - 32:], O0[:, S - 32:]) and torch.equal(l1[:, S - 32:], l0[:, S - 32:])
    assert (O1 - O0).abs().max().item() <= 5e-4
    assert (l1 - l0).abs().max().item() <= 5e-4


@pytest.mark.parametrize("hq,hkv,sq,sk,d,causal", [
    (2, 2, 256, 256, 128, False), (2, 2, 256, 256, 128, True), (4, 2, 160, 224, 128, False),
    (4, 1, 96, 192, 128, True), (2, 2, 192, 320, 64, False), (3, 3, 128, 128, 64, True),
    (2, 1, 1024, 1024, 128, True), (4, 4, 4096, 4096, 64, False), (6, 2, 3840, 3840, 64, True)])
def test_bf16_bwd_fused_dkdv_bit_identical(lib, monkeypatch, hq, hkv, sq, sk, d, causal):
    """The fused dK+dV path (default: dQ recomputes dS), its dS-record variant (dQ reads bf16 dS
    records) and the split dV / dK kernels give identical gradients (same P / dS operands and
    accumulation order; partial workgroups, GQA, Sq != Sk, causal)."""
    from quantizedattention_amd import attention_bf16 as A
    g = torch.Generator().manual_seed(11)
    q = torch.randn((1, hq, sq, d), generator=g).half().cuda()
    k = torch.randn((1, hkv, sk, d), generator=g).half().cuda()
    v = torch.randn((1, hkv, sk, d), generator=g).bfloat16().cuda()
    dO = torch.randn((1, hq, sq, d), generator=g).cuda()
    O, lse = A.helion_atten_bf16_fwd_training(q, k, v, causal)
    monkeypatch.setattr(A, "_BWD_ENTRY", "ws")
    ws = A.helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, causal, dO)
    monkeypatch.setattr(A, "_BWD_ENTRY", "qattn_bf16_bwd_ex")
    fused = A.helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, causal, dO)
    monkeypatch.setattr(A, "_BWD_ENTRY", "qattn_bf16_bwd_split_ex")
    split = A.helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, causal, dO)
    torch.cuda.synchronize()
    for name, a, b, c in zip(("dq", "dk", "dv"), ws, fused, split):
        assert torch.equal(a, b), name
        assert torch.equal(b, c), name


def test_bf16_torch_func_grad(lib):
    """torch.func.grad through FlashAttention_2_BF16_autograd_function (new-style, as bf16:16-85)
    gives the .backward() gradients bit for bit."""
    from quantizedattention_amd.attention_bf16 import flash_atten_2_bf16
    q, k, v = (t.cuda() for t in _inputs((1, 2, 128, 64), seed=23))
    w = torch.randn((1, 2, 128, 64), generator=torch.Generator().manual_seed(24)).cuda()

    def loss(a, b, c):
        return (flash_atten_2_bf16(a, b, c, False) * w).sum()
    g = torch.func.grad(loss, argnums=(0, 1, 2))(q, k, v)
    qd, kd, vd = (t.clone().requires_grad_(True) for t in (q, k, v))
    loss(qd, kd, vd).backward()
    for a, b in zip(g, (qd.grad, kd.grad, vd.grad)):
        assert torch.equal(a, b)
