"""int8 path on the GPU vs the CPU restatement (oracle/restate.py).

Tolerances (stated here):
  * quantisation indices and scales (q, k, v, dO): bit-exact;
  * O: max|O - O_oracle| <= 1e-2 (north star); lse: <= 2 fp16 ulp of |lse| (+1e-3 abs);
  * grads: relL2 vs the corrected oracle <= conftest.INT8_BWD_REL (0.015) and vs fp32 autograd truth <= 0.15.
"""
import pytest
import torch

from conftest import INT8_BWD_REL

from oracle import restate as R

pytestmark = pytest.mark.gpu

SHAPES = [(1, 2, 128, 64), (1, 2, 256, 128), (2, 3, 96, 128), (1, 1, 32, 64), (1, 8, 512, 128)]


def _inputs(shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(shape, generator=g) * scale) for _ in range(3)]


@pytest.mark.parametrize("shape", SHAPES)
def test_int8_fwd_matches_oracle(lib, shape):
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    q, k, v = _inputs(shape)
    qh, kh, vh = q.half(), k.half(), v.half()
    ref = R.int8_fwd(qh, kh, vh)
    out = helion_atten_int8_hl_dot_fwd(qh.cuda(), kh.cuda(), vh.cuda())
    torch.cuda.synchronize()
    names = ["O", "lse", "q_i8", "k_i8T", "v_i8", "sq", "sk", "sv"]
    for i in (2, 3, 4, 5, 6, 7):
        assert torch.equal(out[i].cpu(), ref[i]), f"{names[i]} not bit-exact"
    assert out[8] == ref[8] == 32 and out[9] == ref[9] == 32
    assert out[0].shape == ref[0].shape and out[0].dtype == torch.float16
    err = (out[0].float().cpu() - ref[0].float()).abs().max().item()
    assert err <= 1e-2, err
    lerr = (out[1].float().cpu() - ref[1].float()).abs()
    assert (lerr <= 2 * 2.0 ** -10 * ref[1].float().abs() + 1e-3).all(), lerr.max().item()


def test_int8_quant_edge_cases(lib):
    """All-zero block, tiny values, exact ties and large magnitudes quantise bit-exactly."""
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    B, H, S, D = 1, 1, 128, 64
    q = torch.randn(B, H, S, D)
    q[:, :, :32] = 0                               # all-zero block -> scale 0, idx 0
    q[:, :, 32:64] *= 1e-4                         # subnormal-ish fp16 values
    q[:, :, 64:96] = torch.round(q[:, :, 64:96] * 8) / 8   # many exact ties
    q[:, :, 96:] *= 1000                           # large magnitudes
    k = torch.randn(B, H, S, D)
    v = torch.randn(B, H, S, D)
    ref = R.int8_fwd(q.half(), k.half(), v.half())
    out = helion_atten_int8_hl_dot_fwd(q.half().cuda(), k.half().cuda(), v.half().cuda())
    assert torch.equal(out[2].cpu(), ref[2])
    assert torch.equal(out[5].cpu(), ref[5])


def test_int8_fwd_deterministic(lib):
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    q, k, v = [t.half().cuda() for t in _inputs((1, 4, 256, 128), seed=3)]
    a = helion_atten_int8_hl_dot_fwd(q, k, v)
    b = helion_atten_int8_hl_dot_fwd(q, k, v)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_int8_fwd_large_size_properties(lib):
    """North-star size (4,32,4096,128): finite; constant V reproduces the constant; one head
    checked against the oracle at full length."""
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    B, H, S, D = 4, 32, 4096, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    k = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    v = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    out = helion_atten_int8_hl_dot_fwd(q, k, torch.ones_like(v))
    O = out[0].float()
    assert torch.isfinite(O).all()
    assert (O - 1).abs().max().item() < 0.05  # only the P-trunc bias separates it from 1
    out = helion_atten_int8_hl_dot_fwd(q, k, v)
    b, hh = 1, 5
    ref = R.int8_fwd(q[b:b + 1, hh:hh + 1].cpu(), k[b:b + 1, hh:hh + 1].cpu(),
                     v[b:b + 1, hh:hh + 1].cpu())
    err = (out[0][b, hh].float().cpu() - ref[0][0, 0].float()).abs().max().item()
    assert err <= 1e-2, err


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("shape", [(1, 2, 128, 64), (1, 2, 256, 128), (2, 2, 192, 128), (1, 4, 512, 128)])
def test_int8_bwd_matches_oracle(lib, shape):
    from quantizedattention_amd.attention_int8 import (helion_atten_int8_hl_dot_bwd,
                                                       helion_atten_int8_hl_dot_fwd)
    q, k, v = [t.half() for t in _inputs(shape, seed=31)]
    dO = torch.randn(shape, generator=torch.Generator().manual_seed(32)).half()
    out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda())
    O, lse, qi, kiT, vi, sq, sk, sv, Bq, Bkv = out
    dq, dk, dv = helion_atten_int8_hl_dot_bwd(dO.cuda(), qi, sq, kiT, None, sk, vi, sv, O, lse, Bq, Bkv)
    torch.cuda.synchronize()
    rq, rk, rv = R.int8_bwd(dO, qi.cpu(), sq.cpu(), kiT.cpu(), None, sk.cpu(), vi.cpu(), sv.cpu(),
                            O.cpu(), lse.cpu())
    for name, a, b in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        assert a.dtype == torch.float16 and a.shape == shape
        rel = _rel(a.cpu(), b)
        print(f"RELL2 int8-bwd-vs-oracle {name} {rel:.5f}")
        assert rel <= INT8_BWD_REL, (name, rel)
    tq, tk, tv = R.attention_grads_truth(q, k, v, dO, False)
    for name, a, b in (("dq", dq, tq), ("dk", dk, tk), ("dv", dv, tv)):
        assert _rel(a.cpu(), b) <= 0.15, (name, _rel(a.cpu(), b))


def test_sage_attention_autograd(lib):
    """sage_attention_3_int8 end to end: smoothing forward + corrected int8 backward."""
    from quantizedattention_amd.attention_int8 import (SageAttention3_Int8_autograd_function,
                                                       sage_attention_3_int8)
    shape = (2, 2, 256, 64)
    q, k, v = [t.half() for t in _inputs(shape, seed=41)]
    k = k + 3.0  # a large shared key offset: smoothing removes it without changing softmax
    qd, kd, vd = (t.cuda().requires_grad_(True) for t in (q, k, v))
    out = sage_attention_3_int8(qd, kd, vd)
    outs = SageAttention3_Int8_autograd_function.apply(qd, kd, vd)
    assert len(outs) == 11 and outs[2].shape == (2, 2, 1, 64) and outs[9] == 32
    ks, km = R.k_smooth(k)
    ref = R.int8_fwd(q, ks, v)
    assert (out.float().cpu() - ref[0].float()).abs().max().item() <= 1e-2
    assert torch.equal(outs[2].cpu(), km)
    gt = torch.randn(shape, generator=torch.Generator().manual_seed(42))
    torch.nn.functional.mse_loss(out.float(), gt.cuda()).backward()
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    torch.nn.functional.mse_loss(R.baseline_pytorch_attention(qf, kf, vf, 64, False), gt).backward()
    for a, b in ((qd.grad, qf.grad), (kd.grad, kf.grad), (vd.grad, vf.grad)):
        assert _rel(a.cpu(), b) <= 0.15


def test_quant_image_and_bwd_prep(lib):
    """qattn_int8_quant_img writes bf16(idx) exactly; qattn_int8_bwd_prep (one pass) gives the same
    dO indices/scales as the quantiser, bf16(dO_i8), and LD = {lse, f16(rowsum f16(dO*O))}."""
    from quantizedattention_amd import _lib
    g = torch.Generator().manual_seed(77)
    B, H, S, D = 1, 2, 128, 128
    N = B * H * S
    x = torch.randn((N, D), generator=g).half().cuda()
    O = torch.randn((N, D), generator=g).half().cuda()
    lse = (torch.rand(N, generator=g) * 8).half().cuda()
    P, st = _lib.ptr, _lib.stream_of(x)
    idx = torch.empty((N, D), dtype=torch.int8, device="cuda")
    sc = torch.empty((N // 32,), dtype=torch.float16, device="cuda")
    img = torch.empty((N, D), dtype=torch.bfloat16, device="cuda")
    _lib.call("qattn_int8_quant_img", P(x), P(idx), P(sc), None, P(img), None, N, S, D, st)
    ridx, rsc = R.quant_blocks(x.cpu())
    torch.cuda.synchronize()
    assert torch.equal(idx.cpu(), ridx) and torch.equal(sc.cpu().view(torch.int16), rsc.view(torch.int16))
    assert torch.equal(img.cpu(), ridx.to(torch.bfloat16))
    di = torch.empty_like(idx)
    ds = torch.empty_like(sc)
    dimg = torch.empty_like(img)
    LD = torch.empty((N, 2), dtype=torch.float32, device="cuda")
    _lib.call("qattn_int8_bwd_prep", P(x), P(O), P(lse), P(di), P(ds), P(LD), P(dimg), B * H, S, D, st)
    torch.cuda.synchronize()
    assert torch.equal(di.cpu(), ridx) and torch.equal(ds.cpu().view(torch.int16), rsc.view(torch.int16))
    assert torch.equal(dimg.cpu(), ridx.to(torch.bfloat16))
    Dref = (x.cpu().float() * O.cpu().float()).half().float().sum(-1).half().float()
    assert torch.equal(LD[:, 0].cpu(), lse.cpu().float())
    assert (LD[:, 1].cpu() - Dref).abs().max().item() <= 2 * 2.0 ** -10 * Dref.abs().max().item()


def test_sage_function_new_style(lib):
    """The autograd Function is new-style like the reference (int8:20-65): a direct
    Function.forward(q, k, v) returns the 11-tuple, and torch.func.grad runs through it with the same
    gradients as .backward() (which takes the bf16 images from the forward's quantiser pass; the
    functorch path may rebuild them from q_i8 / k_i8 — bit-identical either way)."""
    from quantizedattention_amd.attention_int8 import (SageAttention3_Int8_autograd_function as F,
                                                       sage_attention_3_int8)
    shape = (1, 2, 128, 128)
    q, k, v = [t.half().cuda() for t in _inputs(shape, seed=51)]
    outs = F.forward(q, k, v)
    assert len(outs) == 11 and outs[9] == 32 and outs[10] == 32
    assert outs[4].shape == (128, 2 * 128) and outs[4].stride() == (1, 128)
    ref = sage_attention_3_int8(q, k, v)
    assert torch.equal(outs[0], ref)
    w = torch.randn(shape, generator=torch.Generator().manual_seed(52)).cuda()

    def loss(q_, k_, v_):
        return (sage_attention_3_int8(q_, k_, v_).float() * w).sum()
    gq, gk, gv = torch.func.grad(loss, argnums=(0, 1, 2))(q, k, v)
    qd, kd, vd = (t.clone().requires_grad_(True) for t in (q, k, v))
    loss(qd, kd, vd).backward()
    assert torch.equal(gq, qd.grad) and torch.equal(gk, kd.grad) and torch.equal(gv, vd.grad)
    from quantizedattention_amd import attention_int8
    assert not attention_int8._IMAGES, "image hand-off entries leaked"


@pytest.mark.parametrize("shape,causal,G", [((1, 2, 256, 128), False, 1), ((2, 4, 160, 64), True, 2),
                                            ((1, 8, 96, 128), False, 4), ((1, 2, 384, 64), False, 1)])
def test_int8_fwd_q_fused_bit_identical(lib, shape, causal, G):
    """qattn_int8_attn_fwd_qf (q quantised in the attention kernel's prologue) equals the separate
    quantiser + qattn_int8_attn_fwd_ex bit for bit: q_i8, sq, the bf16 image, O and lse."""
    from quantizedattention_amd import _lib
    B, H, S, D = shape
    g = torch.Generator().manual_seed(21)
    q = (torch.randn(shape, generator=g) * 3).half().cuda()
    q[0, 0, :32] = 0                                   # an all-zero block (sq = 0)
    k, v = ((torch.randn((B, H // G, S, D), generator=g) * 2).half().cuda() for _ in range(2))
    N, Nkv = B * H * S, B * (H // G) * S
    e = lambda *s_, dt: torch.empty(s_, dtype=dt, device="cuda")  # noqa: E731
    ki, vi, vt = e(Nkv, D, dt=torch.int8), e(Nkv, D, dt=torch.int8), e(Nkv, D, dt=torch.int8)
    sk, sv = e(Nkv // 32, dt=torch.float16), e(Nkv // 32, dt=torch.float16)
    st = _lib.stream_of(q)
    P = _lib.ptr
    _lib.call("qattn_int8_quant", P(k), P(ki), P(sk), None, None, Nkv, S, D, st)
    _lib.call("qattn_int8_quant_vt", P(v), P(vi), P(sv), P(vt), Nkv, D, st)
    qks = float(torch.tensor(1 / D ** 0.5 * 1.44269504, dtype=torch.float32))
    outs = []
    for fused in (False, True):
        qi, sq = e(N, D, dt=torch.int8), e(N // 32, dt=torch.float16)
        qb = e(N, D, dt=torch.bfloat16)
        O, lse = e(N, D, dt=torch.float16), e(N, dt=torch.float16)
        if fused:
            _lib.call("qattn_int8_attn_fwd_qf", P(q), P(qi), P(sq), P(qb), P(ki), P(sk), P(vt), P(sv), P(O),
                      P(lse), B * H, S, S, G, int(causal), D, qks, st)
        else:
            _lib.call("qattn_int8_quant_img", P(q), P(qi), P(sq), None, P(qb), None, N, S, D, st)
            _lib.call("qattn_int8_attn_fwd_ex", P(qi), P(sq), P(ki), P(sk), P(vt), P(sv), P(O), P(lse),
                      B * H, S, S, G, int(causal), D, qks, st)
        outs.append((qi, sq, qb, O, lse))
    torch.cuda.synchronize()
    for a, b_ in zip(*outs):
        assert torch.equal(a.view(torch.uint8) if a.dtype == torch.int8 else a.view(torch.int16),
                           b_.view(torch.uint8) if b_.dtype == torch.int8 else b_.view(torch.int16))


@pytest.mark.parametrize("shape", [(1, 3, 32, 128), (2, 3, 96, 64), (1, 2, 4096, 128), (2, 2, 1056, 128)])
@pytest.mark.parametrize("img", [False, True])
def test_fused_k_smooth_bit_identical(lib, shape, img):
    """qattn_int8_quant_k_smooth (k-mean and the smoothed quantiser in one launch) equals
    qattn_kmean + qattn_int8_quant_img bit for bit: k_mean, k_i8, sk and the bf16 image."""
    from quantizedattention_amd import _lib
    B, H, S, D = shape
    g = torch.Generator(device="cuda").manual_seed(81)
    k = (torch.randn(shape, device="cuda", generator=g) * 3 + 0.5).half()
    N = B * H * S
    st = _lib.stream_of(k)

    def bufs():
        return (torch.empty((B * H, D), dtype=torch.float16, device="cuda"),
                torch.empty((N, D), dtype=torch.int8, device="cuda"),
                torch.empty((N // 32,), dtype=torch.float16, device="cuda"),
                torch.empty((N, D), dtype=torch.bfloat16, device="cuda") if img else None)
    km1, ki1, sk1, kb1 = bufs()
    _lib.call("qattn_kmean", _lib.ptr(k), _lib.ptr(km1), B * H, S, D, st)
    _lib.call("qattn_int8_quant_img", _lib.ptr(k), _lib.ptr(ki1), _lib.ptr(sk1), None, _lib.ptr(kb1),
              _lib.ptr(km1), N, S, D, st)
    km2, ki2, sk2, kb2 = bufs()
    _lib.call("qattn_int8_quant_k_smooth", _lib.ptr(k), _lib.ptr(km2), _lib.ptr(ki2), _lib.ptr(sk2),
              _lib.ptr(kb2), B * H, S, D, st)
    torch.cuda.synchronize()
    assert torch.equal(km1, km2) and torch.equal(ki1, ki2) and torch.equal(sk1, sk2)
    if img:
        assert torch.equal(kb1, kb2)
