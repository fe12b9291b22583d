"""JVP path on the GPU.  Tolerances: O and tO max-abs <= 1e-2 vs
torch.func.jvp of the fp32 baseline on the same (bf16-representable) inputs, and vs the restatement."""
import pytest
import torch

from oracle import restate as R

pytestmark = pytest.mark.gpu


def _inputs(shape, seed, ones_tangent=False):
    g = torch.Generator().manual_seed(seed)
    prim = [torch.randn(shape, generator=g).bfloat16().float() for _ in range(3)]
    if ones_tangent:  # the reference test's tangents (jvp:242-245)
        tan = [torch.ones(shape) for _ in range(3)]
    else:
        tan = [torch.randn(shape, generator=g).bfloat16().float() for _ in range(3)]
    return prim, tan


@pytest.mark.parametrize("shape", [(1, 2, 128, 64), (2, 2, 256, 128), (1, 3, 192, 128)])
@pytest.mark.parametrize("ones", [False, True])
def test_jvp_matches_torch_func_jvp(lib, shape, ones):
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    (q, k, v), (tq, tk, tv) = _inputs(shape, 7, ones)
    O, tO, lse = helion_attention_jvp_forward_fp32(*(t.cuda().bfloat16() for t in (q, k, v, tq, tk, tv)))
    torch.cuda.synchronize()
    Ot, tOt = R.jvp_truth(q, k, v, tq, tk, tv)
    assert (O.cpu() - Ot).abs().max().item() <= 1e-2
    assert (tO.cpu() - tOt).abs().max().item() <= 1e-2 * max(1.0, tOt.abs().max().item() / 10)
    Or, tOr, lser = R.jvp_fwd(q, k, v, tq, tk, tv)
    assert (lse.cpu() - lser).abs().max().item() <= 1e-2


@pytest.mark.parametrize("shape", [(1, 2, 128, 64), (2, 2, 256, 128), (1, 3, 96, 128)])
def test_jvp_fp32_mode(lib, shape):
    """fp32 inputs run the split-bf16 (hi*hi + hi*lo + lo*hi + lo*lo) kernel: SURVEY §8c fp32 mode, <= 1e-5
    vs torch.func.jvp of the fp32 baseline (tO relative to its magnitude)."""
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    g = torch.Generator().manual_seed(11)
    q, k, v, tq, tk, tv = (torch.randn(shape, generator=g) for _ in range(6))
    O, tO, lse = helion_attention_jvp_forward_fp32(*(t.cuda() for t in (q, k, v, tq, tk, tv)))
    torch.cuda.synchronize()
    Ot, tOt = R.jvp_truth(q, k, v, tq, tk, tv)
    assert (O.cpu() - Ot).abs().max().item() <= 1e-5
    assert (tO.cpu() - tOt).abs().max().item() <= 1e-5 * max(1.0, tOt.abs().max().item())
    _, _, lser = R.jvp_fwd(q, k, v, tq, tk, tv)
    assert (lse.cpu() - lser).abs().max().item() <= 1e-5 * max(1.0, lser.abs().max().item())


def test_split_bf16_exact(lib):
    from quantizedattention_amd import _lib
    x = torch.randn(4096, generator=torch.Generator().manual_seed(3)).cuda()
    hi = torch.empty(4096, dtype=torch.bfloat16, device="cuda")
    lo = torch.empty_like(hi)
    _lib.call("qattn_split_bf16", _lib.ptr(x), _lib.ptr(hi), _lib.ptr(lo), 4096, _lib.stream_of(x))
    torch.cuda.synchronize()
    hr = x.cpu().bfloat16()
    lr = (x.cpu() - hr.float()).bfloat16()
    assert torch.equal(hi.cpu().view(torch.int16), hr.view(torch.int16))
    assert torch.equal(lo.cpu().view(torch.int16), lr.view(torch.int16))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_jvp_autograd_function_forward_mode(lib, dtype):
    """torch.func.jvp and forward_ad dual tensors route to the HIP tangent kernel."""
    import torch.autograd.forward_ad as fwAD
    from quantizedattention_amd.attention_jvp import attention_jvp, helion_attention_jvp_forward_fp32
    g = torch.Generator().manual_seed(5)
    shape = (1, 2, 128, 64)
    q, k, v, tq, tk, tv = (torch.randn(shape, generator=g).to(dtype).cuda() for _ in range(6))
    from quantizedattention_amd import attention_jvp as J
    O_ref, tO_ref, _ = helion_attention_jvp_forward_fp32(q, k, v, tq, tk, tv)
    J.LAUNCHES.update(primal=0, tangent=0)
    O, tO = torch.func.jvp(attention_jvp, (q, k, v), (tq, tk, tv))
    torch.cuda.synchronize()
    assert torch.equal(O, O_ref) and torch.equal(tO, tO_ref)
    # one launch per call: the forward defers O to the tangent kernel, which computes O and tO
    assert J.LAUNCHES == {"primal": 0, "tangent": 1}, J.LAUNCHES
    with fwAD.dual_level():
        dq = fwAD.make_dual(q, tq)
        dk = fwAD.make_dual(k, tk)
        dv = fwAD.make_dual(v, tv)
        out = attention_jvp(dq, dk, dv)
        p, t = fwAD.unpack_dual(out)
    assert torch.equal(p, O_ref) and torch.equal(t, tO_ref)
    assert J.LAUNCHES == {"primal": 0, "tangent": 2}, J.LAUNCHES
    # plain calls (no tangent anywhere) run the primal-only kernel; so do other transforms
    assert torch.equal(attention_jvp(q, k, v), O_ref)
    assert J.LAUNCHES == {"primal": 1, "tangent": 2}, J.LAUNCHES
    with fwAD.dual_level():   # a dual on one input only: the other tangents are zeros
        out = attention_jvp(fwAD.make_dual(q, tq), k, v)
        p1, t1 = fwAD.unpack_dual(out)
    O1, tO1, _ = helion_attention_jvp_forward_fp32(q, k, v, tq, torch.zeros_like(k), torch.zeros_like(v))
    assert torch.equal(p1, O1) and torch.equal(t1, tO1)
    assert J.LAUNCHES["primal"] == 1 and not getattr(J._DEFER, "pending", [])
    # matches forward-mode AD of the fp32 baseline within the mode's tolerance
    Ot, tOt = R.jvp_truth(*(x.float().cpu() for x in (q, k, v, tq, tk, tv)))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert (O.cpu() - Ot).abs().max().item() <= tol
    assert (tO.cpu() - tOt).abs().max().item() <= tol * max(1.0, tOt.abs().max().item())


def test_jvp_constant_inputs_under_transform(lib):
    """attention_jvp on inputs that carry no tangent at the current torch.func.jvp level
    (the primal of the transformed function is something else) must return the real O, not the
    deferred forward's empty buffer, and leave no pending entry behind."""
    from quantizedattention_amd import attention_jvp as J
    from quantizedattention_amd.attention_jvp import attention_jvp, helion_attention_jvp_forward_fp32
    g = torch.Generator().manual_seed(9)
    shape = (1, 2, 64, 64)
    q0, k0, v0 = (torch.randn(shape, generator=g).cuda() for _ in range(3))
    x, tx = (torch.randn(shape, generator=g).cuda() for _ in range(2))
    O_ref, _, _ = helion_attention_jvp_forward_fp32(q0, k0, v0, *(torch.zeros_like(q0),) * 3)
    for _ in range(3):   # repeated calls: a stale entry would be matched by reused addresses
        y, ty = torch.func.jvp(lambda a: attention_jvp(q0, k0, v0) + a, (x,), (tx,))
        torch.cuda.synchronize()
        assert torch.equal(y, O_ref + x)
        assert torch.equal(ty, tx)
        assert not getattr(J._DEFER, "pending", [])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(1, 4, 2, 128, 128, 128), (2, 6, 3, 64, 192, 64)])
def test_jvp_grouped_query(lib, dtype, shape):
    """Grouped-query JVP (extension): query head h reads key/value head h // G.
    Bit-identical to the same call with k, v, tk, tv expanded to every query head, and within the
    mode's tolerance of torch.func.jvp on the expanded fp32 problem ("parity unpinned": the
    reference's JVP kernel has no grouped shapes)."""
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    B, H, Hkv, Sq, Sk, D = shape
    g = torch.Generator().manual_seed(11)
    q, tq = (torch.randn((B, H, Sq, D), generator=g) for _ in range(2))
    k, v, tk, tv = (torch.randn((B, Hkv, Sk, D), generator=g) for _ in range(4))
    dev = lambda t: t.to(dtype).cuda()  # noqa: E731
    rep = lambda t: t.repeat_interleave(H // Hkv, dim=1)  # noqa: E731
    O, tO, lse = helion_attention_jvp_forward_fp32(dev(q), dev(k), dev(v), dev(tq), dev(tk), dev(tv))
    Oe, tOe, lsee = helion_attention_jvp_forward_fp32(dev(q), dev(rep(k)), dev(rep(v)), dev(tq),
                                                      dev(rep(tk)), dev(rep(tv)))
    torch.cuda.synchronize()
    assert torch.equal(O, Oe) and torch.equal(tO, tOe) and torch.equal(lse, lsee)
    f = lambda a, b, c: torch.softmax(a @ b.transpose(-1, -2) / D ** 0.5, -1) @ c  # noqa: E731
    qr, kr, vr = (t.to(dtype).double() for t in (q, rep(k), rep(v)))
    tqr, tkr, tvr = (t.to(dtype).double() for t in (tq, rep(tk), rep(tv)))
    Or, tOr = torch.func.jvp(f, (qr, kr, vr), (tqr, tkr, tvr))
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert (O.cpu().double() - Or).abs().max().item() <= tol
    scale = max(1.0, tOr.abs().max().item())
    assert (tO.cpu().double() - tOr).abs().max().item() <= tol * scale


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape", [(2, 4, 2, 256, 192, 128), (1, 2, 2, 96, 128, 64)])
def test_jvp_primal_only_bit_identical(lib, dtype, shape):
    """The primal-only kernel (the N1 Function's forward when no tangent follows) returns the tangent
    kernel's O and lse bit for bit."""
    from quantizedattention_amd.attention_jvp import _jvp
    B, H, Hkv, Sq, Sk, D = shape
    g = torch.Generator().manual_seed(13)
    q, tq = (torch.randn((B, H, Sq, D), generator=g).to(dtype).cuda() for _ in range(2))
    k, v, tk, tv = (torch.randn((B, Hkv, Sk, D), generator=g).to(dtype).cuda() for _ in range(4))
    O, tO, lse = _jvp(q, k, v, (tq, tk, tv))
    Op, none, lsep = _jvp(q, k, v, None)
    torch.cuda.synchronize()
    assert none is None
    assert torch.equal(O, Op) and torch.equal(lse, lsep)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_jvp_non_contiguous_inputs(lib, dtype):
    """q/k/v and tangents made by transposing [B,S,H,D] tensors (non-contiguous): every contiguous
    copy must outlive the launch that reads it.  Bit-identical to the call on contiguous copies, for
    the tangent kernel and the primal-only kernel."""
    from quantizedattention_amd.attention_jvp import _jvp
    g = torch.Generator().manual_seed(17)
    B, S, H, D = 2, 192, 3, 64
    xs = [torch.randn((B, S, H, D), generator=g).to(dtype).cuda().transpose(1, 2) for _ in range(6)]
    assert not any(x.is_contiguous() for x in xs)
    ys = [x.contiguous() for x in xs]
    O, tO, lse = _jvp(*xs[:3], tuple(xs[3:]))
    Oc, tOc, lsec = _jvp(*ys[:3], tuple(ys[3:]))
    Op, _, lsep = _jvp(*xs[:3], None)
    torch.cuda.synchronize()
    assert torch.equal(O, Oc) and torch.equal(tO, tOc) and torch.equal(lse, lsec)
    assert torch.equal(Op, Oc) and torch.equal(lsep, lsec)


def test_jvp_deferred_forward_without_jvp_rule(lib, monkeypatch):
    """A call that defers its O to the jvp rule (attention_jvp saw a tangent coming) but whose jvp
    rule never runs gets O from the primal kernel, and leaves no deferred entry behind."""
    from quantizedattention_amd import attention_jvp as J
    g = torch.Generator(device="cuda").manual_seed(11)
    q, k, v = (torch.randn((1, 2, 128, 64), device="cuda", generator=g).bfloat16() for _ in range(3))
    plain = J.attention_jvp(q, k, v)          # no transform: the primal kernel
    monkeypatch.setattr(J, "_jvp_follows", lambda tensors: True)
    deferred = J.attention_jvp(q, k, v)       # deferred, and no jvp rule follows
    torch.cuda.synchronize()
    assert torch.equal(deferred, plain)
    assert not getattr(J._DEFER, "pending", [])
    assert not getattr(J._DEFER, "on", False)
