"""MX-FP4 inference forward on the GPU against oracle/mxfp4.py.

Quantisers: bit-exact (packed nibbles and e8m0 bytes).  Attention: the kernel computes the same
definition with the hardware exp2 (v_exp_f32) and MFMA summation order, so a P element that sits
on an e2m1 rounding boundary may land on the neighbouring code: O within 2e-2 max-abs and 2e-3
relative L2 of the oracle, lse within 1e-4.  Parity with the reference is unpinned (it has no FP4
kernel); tests/test_mxfp4_oracle.py bounds the definition against fp32 attention.
"""
import pytest
import torch

from oracle import mxfp4 as M
from oracle import restate as R

pytestmark = pytest.mark.gpu

# (B, Hq, Hkv, Sq, Sk)
SHAPES = [(1, 2, 2, 128, 128), (2, 4, 2, 96, 256), (1, 2, 1, 160, 320)]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


def test_quant_rows_bit_exact(lib):
    from quantizedattention_amd.attention_mxfp4 import mxfp4_quantize_rows
    g = torch.Generator().manual_seed(0)
    x = torch.randn((256, 128), generator=g) * torch.logspace(-6, 4, 256)[:, None]
    x = x.clamp(-65504, 65504).half()
    x[0] = 0.0                                   # zero block -> scale byte 0
    x[1, :32] = -0.0
    x[2, 5] = 65504.0                            # largest fp16
    x[3] = 2.0 ** -24                            # fp16 subnormals
    for D in (128, 64):
        xd = x.reshape(-1, D)
        q4, sc = mxfp4_quantize_rows(xd.cuda())
        r4, rs = M.quant_rows(xd)
        assert torch.equal(sc.cpu(), rs), D
        assert torch.equal(q4.cpu(), r4), D


def test_quant_rows_smoothed_bit_exact(lib):
    """k smoothing inside the quantiser: rows of head i become f16(k - k_mean[i]) first."""
    from quantizedattention_amd import _lib
    from quantizedattention_amd.attention_mxfp4 import mxfp4_quantize_rows
    g = torch.Generator().manual_seed(5)
    k = (torch.randn((2, 3, 96, 128), generator=g) + 4.0).half()
    kc = k.cuda()
    km = torch.empty((2, 3, 1, 128), dtype=torch.float16, device="cuda")
    _lib.call("qattn_kmean", _lib.ptr(kc), _lib.ptr(km), 6, 96, 128, _lib.stream_of(kc))
    q4, sc = mxfp4_quantize_rows(kc, km)
    ks = (k.float() - km.cpu().float()).half()
    r4, rs = M.quant_rows(ks.reshape(-1, 128))
    assert torch.equal(sc.cpu(), rs) and torch.equal(q4.cpu(), r4)


def test_quant_v_bit_exact(lib):
    from quantizedattention_amd.attention_mxfp4 import mxfp4_quantize_v
    g = torch.Generator().manual_seed(1)
    v = (torch.randn((2, 3, 192, 128), generator=g) * 3).half()
    v[0, 0, :64, 7] = 0.0
    vt, vs = mxfp4_quantize_v(v.cuda())
    rt, rs = M.quant_vt(v.reshape(6, 192, 128))
    assert torch.equal(vs.cpu(), rs) and torch.equal(vt.cpu(), rt)


@pytest.mark.parametrize("shape", SHAPES)
def test_mxfp4_fwd_vs_oracle(lib, shape):
    from quantizedattention_amd.attention_mxfp4 import mxfp4_attn_fwd
    B, H, Hkv, Sq, Sk = shape
    g = torch.Generator().manual_seed(2)
    q = torch.randn((B, H, Sq, 128), generator=g).half()
    k = torch.randn((B, Hkv, Sk, 128), generator=g).half()
    v = torch.randn((B, Hkv, Sk, 128), generator=g).half()
    O, lse, ops = mxfp4_attn_fwd(q.cuda(), k.cuda(), v.cuda(), smooth_k=False)
    torch.cuda.synchronize()
    RO, Rl, rops = M.mxfp4_fwd(q, k, v)
    for a, b in zip(ops, rops):
        assert torch.equal(a.cpu().reshape(b.shape), b)
    assert O.shape == (B, H, Sq, 128) and lse.shape == (B * H, Sq)
    err = (O.float().cpu() - RO.float()).abs().max().item()
    assert err <= 2e-2, err
    assert _rel(O.cpu(), RO) <= 2e-3, _rel(O.cpu(), RO)
    assert (lse.cpu() - Rl).abs().max().item() <= 1e-4


def test_mxfp4_uniform_keys(lib):
    """k = 0: P = 1 exactly for every key, so O is the mean of the dequantised V rows."""
    from quantizedattention_amd.attention_mxfp4 import mxfp4_attn_fwd
    g = torch.Generator().manual_seed(3)
    q = torch.randn((1, 2, 64, 128), generator=g).half()
    v = torch.randn((1, 2, 256, 128), generator=g).half()
    O, lse, ops = mxfp4_attn_fwd(q.cuda(), torch.zeros_like(v).cuda(), v.cuda(), smooth_k=False)
    vd = M.deq_vt(ops[4].cpu(), ops[5].cpu()).float().mean(1)          # [2, 128]
    assert (O.float().cpu()[0] - vd[:, None, :]).abs().max().item() <= 1e-3
    assert torch.allclose(lse.cpu(), torch.full((2, 64), 8.0), atol=1e-5)


def test_sage_attention_3_fp4_accuracy(lib):
    """End-to-end with k smoothing, vs exact fp32 attention (the definition's accuracy bound)."""
    from quantizedattention_amd.attention_mxfp4 import sage_attention_3_fp4
    g = torch.Generator().manual_seed(4)
    q = torch.randn((2, 4, 256, 128), generator=g).half()
    k = (torch.randn((2, 4, 512, 128), generator=g) + 2.0).half()   # a large shared key offset
    v = torch.randn((2, 4, 512, 128), generator=g).half()
    O = sage_attention_3_fp4(q.cuda(), k.cuda(), v.cuda())
    ref = R.baseline_pytorch_attention(q.float(), k.float(), v.float(), 128, False)
    cos = torch.nn.functional.cosine_similarity(O.float().cpu().flatten(), ref.flatten(), 0).item()
    assert cos >= 0.95, cos


def test_mxfp4_rejects_bad_shapes(lib):
    from quantizedattention_amd import _lib
    from quantizedattention_amd.attention_mxfp4 import mxfp4_attn_fwd
    q = torch.zeros((1, 2, 64, 128), dtype=torch.float16, device="cuda")
    with pytest.raises(_lib.QAttnError):
        mxfp4_attn_fwd(q, q[:, :, :48], q[:, :, :48])        # Sk % 64
    with pytest.raises(_lib.QAttnError):
        mxfp4_attn_fwd(q[..., :64], q[..., :64], q[..., :64])  # head_dim 64 (quantiser only)
