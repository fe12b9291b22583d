"""int8 path with the generalised shapes of SURVEY §8f N2 (extensions with no reference
counterpart): grouped-query attention (Hq a multiple of Hkv), Sq != Sk and causal masking, against
the oracle's restatement of the same extension (oracle/restate.py int8_fwd / int8_bwd).

Tolerances as tests/test_gpu_int8.py: quantisation bit-exact; O max-abs <= 1e-2 on every row
(causal rows that keep only a few keys included: on the tiles crossing the diagonal the kernel's P_i8
follows the reference chain literally); lse <= 2 fp16 ulp (+1e-3); grads relL2 <= conftest.INT8_BWD_REL (0.015) vs the
oracle.  Parity with the reference is not defined here (the
reference has no such shapes): the oracle pins the documented semantics.
"""
import pytest
import torch

from conftest import INT8_BWD_REL

from oracle import restate as R

pytestmark = pytest.mark.gpu

# (B, Hq, Hkv, Sq, Sk, D)
SHAPES = [(1, 4, 2, 128, 96, 64), (2, 4, 1, 64, 160, 128), (1, 2, 2, 160, 128, 128),
          (1, 2, 2, 128, 128, 64)]


def _inputs(shape, seed=0):
    B, Hq, Hkv, Sq, Sk, D = shape
    g = torch.Generator().manual_seed(seed)
    q = torch.randn((B, Hq, Sq, D), generator=g).half()
    k = torch.randn((B, Hkv, Sk, D), generator=g).half()
    v = torch.randn((B, Hkv, Sk, D), generator=g).half()
    return q, k, v


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("shape", SHAPES + [(1, 8, 8, 256, 256, 128), (1, 4, 2, 96, 224, 64)])
@pytest.mark.parametrize("causal", [False, True])
def test_int8_fwd_gqa_causal(lib, shape, causal):
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    q, k, v = _inputs(shape, seed=1)
    ref = R.int8_fwd(q, k, v, causal=causal)
    out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda(), causal=causal)
    torch.cuda.synchronize()
    for i in (2, 3, 4, 5, 6, 7):
        assert out[i].shape == ref[i].shape and torch.equal(out[i].cpu(), ref[i]), i
    assert out[0].shape == ref[0].shape
    diff = (out[0].float().cpu() - ref[0].float()).abs()
    err = diff.max().item()
    assert err <= 1e-2, err
    lerr = (out[1].float().cpu() - ref[1].float()).abs()
    assert (lerr <= 2 * 2.0 ** -10 * ref[1].float().abs() + 1e-3).all(), lerr.max().item()


def test_int8_causal_first_row_is_first_value(lib):
    """Causal row 0 keeps key 0 only: O[0] is the dequantised v[0] = v_i8[0] * sv (P_i8 = 127,
    sp = 1/127), up to the fp16 roundings of the two P.V operands."""
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    q, k, v = _inputs((1, 2, 2, 64, 64, 64), seed=2)
    out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda(), causal=True)
    O = out[0].float().cpu()
    vi, sv = out[4].cpu().view(2, 64, 64), out[7].float().cpu().view(2, 2)
    vdq0 = vi[:, 0].float() * sv[:, 0:1]                  # head h, row 0, block 0 scale
    assert (O[0, :, 0] - vdq0).abs().max().item() <= 2e-3 * max(1.0, vdq0.abs().max().item())


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("causal", [False, True])
def test_int8_bwd_gqa_causal(lib, shape, causal):
    from quantizedattention_amd.attention_int8 import (helion_atten_int8_hl_dot_bwd,
                                                       helion_atten_int8_hl_dot_fwd)
    B, Hq, Hkv, Sq, Sk, D = shape
    q, k, v = _inputs(shape, seed=3)
    dO = torch.randn((B, Hq, Sq, D), generator=torch.Generator().manual_seed(4)).half()
    O, lse, qi, kiT, vi, sq, sk, sv, Bq, Bkv = helion_atten_int8_hl_dot_fwd(
        q.cuda(), k.cuda(), v.cuda(), causal=causal)
    dq, dk, dv = helion_atten_int8_hl_dot_bwd(dO.cuda(), qi, sq, kiT, None, sk, vi, sv, O, lse, Bq, Bkv,
                                              causal=causal, kv_heads=Hkv)
    torch.cuda.synchronize()
    rq, rk, rv = R.int8_bwd(dO, qi.cpu(), sq.cpu(), kiT.cpu(), None, sk.cpu(), vi.cpu(), sv.cpu(),
                            O.cpu(), lse.cpu(), causal=causal, kv_heads=Hkv)
    assert dq.shape == (B, Hq, Sq, D) and dk.shape == (B, Hkv, Sk, D) and dv.shape == dk.shape
    for name, a, b in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        assert torch.isfinite(a).all(), name
        rel = _rel(a.cpu(), b)
        print(f"RELL2 int8-bwd-vs-oracle {name} {rel:.5f}")
        assert rel <= INT8_BWD_REL, (name, rel)


def test_int8_autograd_gqa_causal(lib):
    """sage_attention_3_int8(..., causal=True) through autograd with 4 query heads per key/value
    head: grads land on the leaves with their own shapes and match the composed oracle."""
    from quantizedattention_amd.attention_int8 import sage_attention_3_int8
    shape = (1, 4, 1, 96, 128, 64)
    q, k, v = _inputs(shape, seed=5)
    qc, kc, vc = (t.cuda().requires_grad_() for t in (q, k, v))
    O = sage_attention_3_int8(qc, kc, vc, causal=True)
    dO = torch.randn(O.shape, generator=torch.Generator().manual_seed(6)).half()
    O.backward(dO.cuda())
    assert qc.grad.shape == q.shape and kc.grad.shape == k.shape and vc.grad.shape == v.shape
    ks, km = R.k_smooth(k)
    ref = R.int8_fwd(q, ks, v, causal=True)
    diff = (O.detach().float().cpu() - ref[0].float()).abs()
    assert diff.max().item() <= 1e-2, diff.max().item()
    rq, rk, rv = R.int8_bwd(dO, ref[2], ref[5], ref[3], km, ref[6], ref[4], ref[7], ref[0], ref[1],
                            causal=True)
    for name, a, b in (("dq", qc.grad, rq), ("dk", kc.grad, rk), ("dv", vc.grad, rv)):
        rel = _rel(a.cpu(), b)
        print(f"RELL2 int8-bwd-vs-oracle {name} {rel:.5f}")
        assert rel <= INT8_BWD_REL, (name, rel)


@pytest.mark.parametrize("shape", SHAPES + [(1, 2, 2, 256, 512, 128), (2, 3, 3, 96, 96, 128)])
@pytest.mark.parametrize("causal", [False, True])
def test_int8_bwd_ws_bit_identical(lib, shape, causal):
    """dQ from the dS workspace written by the fused dK+dV kernel (qattn_int8_attn_bwd_ws) against
    the recomputing dQ kernel (qattn_int8_attn_bwd_ex): same dS_i8 and scales, same operand and MFMA
    order, so dq, dk, dv agree bit for bit -- over GQA, Sq != Sk, causal and partial workgroups."""
    from quantizedattention_amd.attention_int8 import _int8_backward, helion_atten_int8_hl_dot_fwd
    B, Hq, Hkv, Sq, Sk, D = shape
    q, k, v = _inputs(shape, seed=5)
    dO = torch.randn((B, Hq, Sq, D), generator=torch.Generator().manual_seed(6)).half().cuda()
    O, lse, qi, kiT, vi, sq, sk, sv, _, _ = helion_atten_int8_hl_dot_fwd(
        q.cuda(), k.cuda(), v.cuda(), causal=causal)
    a = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, causal=causal, kv_heads=Hkv, use_ws=True)
    b = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, causal=causal, kv_heads=Hkv, use_ws=False)
    torch.cuda.synchronize()
    for name, x, y in zip(("dq", "dk", "dv"), a, b):
        assert torch.isfinite(x).all(), name
        assert torch.equal(x, y), (name, (x.float() - y.float()).abs().max().item())


def test_int8_bwd_ws_bit_identical_large(lib):
    """The same bit-identity at a long sequence, (1, 8, 4096, 128): 128 key tiles per head, every
    workspace record written by a different (key tile, query tile) pair of waves."""
    from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward
    g = torch.Generator(device="cuda").manual_seed(7)
    q, k, v = (torch.randn((1, 8, 4096, 128), device="cuda", generator=g).half() for _ in range(3))
    dO = (torch.randn((1, 8, 4096, 128), device="cuda", generator=g) * 1e-3).half()
    O, lse, qi, kiT, vi, sq, sk, sv, _, qb, kb = _int8_forward(q, k, v, smooth=True, images=True)
    a = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, use_ws=True)
    b = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, use_ws=False)
    torch.cuda.synchronize()
    for name, x, y in zip(("dq", "dk", "dv"), a, b):
        assert torch.isfinite(x).all() and x.abs().max().item() > 0, name
        assert torch.equal(x, y), name


@pytest.mark.parametrize("shape,causal", [((2, 6, 6, 3840, 3840, 64), False), ((2, 8, 2, 1024, 1024, 64), True),
                                          ((2, 6, 6, 4096, 4096, 64), True)])
def test_int8_bwd_ws_long_d64(lib, shape, causal):
    """Long sequences at D = 64, where the dS record store of the last query tile was once followed
    directly by a VALU write of its data register (a store-data hazard hipcc did not pad for an
    SGPR soffset): dword 0 of some records came out wrong, run-dependently, and dq of that tile's
    first 8 rows with it.  Four record runs against the recomputing backward, bit for bit."""
    from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward
    B, Hq, Hkv, Sq, Sk, D = shape
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn((B, Hq, Sq, D), device="cuda", generator=g).half()
    k, v = (torch.randn((B, Hkv, Sk, D), device="cuda", generator=g).half() for _ in range(2))
    dO = torch.randn((B, Hq, Sq, D), device="cuda", generator=g).half()
    O, lse, qi, kiT, vi, sq, sk, sv, _, qb, kb = _int8_forward(q, k, v, smooth=True, images=True, causal=causal)
    kw = dict(causal=causal, kv_heads=Hkv, ws_chunk=0)
    ref = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, use_ws=False, **kw)
    for poison in (None, 0x00, 0x7F, 0x81):
        out = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, use_ws=True, ws_poison=poison, **kw)
        torch.cuda.synchronize()
        for name, a, b in zip(("dq", "dk", "dv"), out, ref):
            assert torch.equal(a, b), (name, poison, int((a != b).sum()))


@pytest.mark.parametrize("shape,causal", [((2, 6, 3, 256, 256, 64), True), ((1, 8, 2, 512, 512, 128), True),
                                          ((2, 4, 4, 256, 256, 128), False)])
def test_int8_bwd_run_to_run_identical(lib, shape, causal):
    """The record backward repeated 8 times gives bit-identical dq, dk, dv (no atomics, one writer
    per record and output tile): a guard against ring / wait-count races, which show up as
    run-to-run differences (tools/race_check.py)."""
    from quantizedattention_amd.attention_int8 import _int8_backward, helion_atten_int8_hl_dot_fwd
    B, Hq, Hkv, Sq, Sk, D = shape
    q, k, v = _inputs(shape, seed=9)
    dO = torch.randn((B, Hq, Sq, D), generator=torch.Generator().manual_seed(10)).half().cuda()
    O, lse, qi, kiT, vi, sq, sk, sv, _, _ = helion_atten_int8_hl_dot_fwd(
        q.cuda() * 2, k.cuda() * 2, v.cuda(), causal=causal)
    ref = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, causal=causal, kv_heads=Hkv, use_ws=True)
    for _ in range(7):
        out = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, causal=causal, kv_heads=Hkv, use_ws=True)
        for name, a, b in zip(("dq", "dk", "dv"), out, ref):
            assert torch.equal(a, b), name


@pytest.mark.parametrize("shape,causal,chunk", [
    ((2, 6, 3, 96, 96, 64), True, None), ((2, 6, 3, 160, 224, 64), False, 1),
    ((1, 8, 2, 288, 288, 128), True, None), ((2, 4, 2, 416, 416, 128), False, 1),
    ((1, 4, 4, 128, 384, 128), False, 2)])
def test_int8_bwd_records_independent_of_workspace_contents(lib, shape, causal, chunk):
    """The dS-record protocol, deterministically: the record backward runs twice, into workspaces
    filled with 0x00 and with 0x7F before the launch, and once without records.  A dQ pass that read
    a record the dK+dV pass had not written would see the fill pattern, so dq (and dk, dv) would
    differ on the first run -- no repetition needed.  GQA, causal, Sq != Sk, partial workgroups
    (Sq not a multiple of the 256-row dK+dV / dQ workgroups), one-pass and head-chunked records."""
    from quantizedattention_amd.attention_int8 import _int8_backward, helion_atten_int8_hl_dot_fwd
    B, Hq, Hkv, Sq, Sk, D = shape
    g = torch.Generator().manual_seed(21)
    q = torch.randn((B, Hq, Sq, D), generator=g)
    k, v = (torch.randn((B, Hkv, Sk, D), generator=g) for _ in range(2))
    dO = torch.randn((B, Hq, Sq, D), generator=g).half().cuda()
    O, lse, qi, kiT, vi, sq, sk, sv, _, _ = helion_atten_int8_hl_dot_fwd(
        q.cuda(), k.cuda(), v.cuda(), causal=causal)
    kw = dict(causal=causal, kv_heads=Hkv, ws_chunk=chunk)
    a = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, use_ws=True, ws_poison=0x00, **kw)
    b = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, use_ws=True, ws_poison=0x7F, **kw)
    c = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, use_ws=False, **kw)
    torch.cuda.synchronize()
    for name, x, y, z in zip(("dq", "dk", "dv"), a, b, c):
        assert torch.isfinite(x).all() and x.abs().max().item() > 0, name
        assert torch.equal(x, y), (name, "depends on the workspace fill")
        assert torch.equal(x, z), (name, "records differ from recomputation")


@pytest.mark.parametrize("i", range(16))
def test_int8_bwd_records_consistency_fuzz(lib, i):
    """Seeded random shapes up to 3072 tokens (grouped heads, Sq != Sk, D 64 / 128, causal or not,
    partial workgroups): the record backward, over two workspace fills and two chunkings, equals the
    recomputing backward bit for bit.  Exact agreement catches what a relL2 bar cannot -- a few
    wrong rows (the store-data hazard of DESIGN.md §4 moved 8 rows of one tile per head)."""
    from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward
    g = torch.Generator().manual_seed(4000 + i)
    pick = lambda xs: xs[int(torch.randint(len(xs), (1,), generator=g))]  # noqa: E731
    D, Hkv, G, B = pick([64, 128]), pick([1, 2, 3]), pick([1, 2, 4]), pick([1, 2])
    Sk = 32 * int(torch.randint(1, 97, (1,), generator=g))
    Sq = Sk if i % 2 else 32 * int(torch.randint(1, 97, (1,), generator=g))
    causal = bool(i % 3 == 0) and Sq <= Sk
    gd = torch.Generator(device="cuda").manual_seed(5000 + i)
    q = torch.randn((B, Hkv * G, Sq, D), device="cuda", generator=gd).half()
    k, v = (torch.randn((B, Hkv, Sk, D), device="cuda", generator=gd).half() for _ in range(2))
    dO = torch.randn((B, Hkv * G, Sq, D), device="cuda", generator=gd).half()
    O, lse, qi, kiT, vi, sq, sk, sv, _, qb, kb = _int8_forward(q, k, v, smooth=True, images=True, causal=causal)
    kw = dict(causal=causal, kv_heads=Hkv)
    ref = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, use_ws=False, **kw)
    for poison, chunk in ((0x00, 0), (0x7F, 1)):
        out = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, use_ws=True, ws_poison=poison,
                             ws_chunk=chunk, **kw)
        torch.cuda.synchronize()
        for name, a, b in zip(("dq", "dk", "dv"), out, ref):
            assert torch.isfinite(a).all(), name
            assert torch.equal(a, b), (name, (B, Hkv * G, Hkv, Sq, Sk, D, causal), poison, chunk)
