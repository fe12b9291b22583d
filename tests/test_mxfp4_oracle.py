"""CPU checks of the MX-FP4 restatement (oracle/mxfp4.py).

The reference has no FP4 kernel, so parity with it is unpinned; these tests pin the restatement to
the OCP MX definition it claims (rounding ties, scale choice, exact round trips of representable
blocks, the V operand key order) and bound its accuracy against exact fp32 attention.
"""
import torch

from oracle import mxfp4 as M
from oracle import restate as R


def test_e2m1_round_to_nearest_even_and_saturation():
    y = torch.tensor([0.25, 0.75, 1.25, 1.75, 2.5, 3.5, 5.0, 7.0, 100.0, 0.2, 0.3, -0.25, -5.0, -0.0])
    got = M.decode(M.rne_e2m1(y))
    want = torch.tensor([0, 1, 1, 2, 2, 4, 4, 6, 6, 0, 0.5, -0.0, -4, -0.0], dtype=torch.float64)
    assert torch.equal(got, want)
    assert torch.equal(torch.signbit(got), torch.signbit(want))
    assert M.rne_e2m1(torch.tensor([-0.25]))[0].item() == 8   # sign kept on a zero result


def test_e8m0_scale_choice():
    amax = torch.tensor([1.0, 6.0, 7.99, 8.0, 0.0, 2.0 ** -20, 65504.0])
    want = torch.tensor([125, 127, 127, 128, 0, 127 - 22, 127 + 15 - 2])
    assert torch.equal(M.e8m0(amax), want)
    # the block maximum lands in [4, 8) after scaling
    b = M.e8m0(amax[amax > 0])
    r = amax[amax > 0].double() / M.scale_value(b)
    assert ((r >= 4) & (r < 8)).all()


def _representable_rows(rows, D, g):
    """fp16 rows whose every 32-block holds grid values times 2^f with one element at +-6 * 2^f."""
    codes = torch.randint(0, 16, (rows, D), generator=g)
    f = torch.randint(-6, 4, (rows, D // 32), generator=g).double()
    x = M.decode(codes).reshape(rows, D // 32, 32)
    x[..., 0] = 6.0 * torch.where(torch.rand((rows, D // 32), generator=g) < 0.5, -1.0, 1.0)
    return (x * torch.pow(2.0, f)[..., None]).reshape(rows, D).half()


def test_rows_round_trip_exact():
    g = torch.Generator().manual_seed(0)
    x = _representable_rows(64, 128, g)
    q4, sc = M.quant_rows(x)
    assert q4.shape == (64, 64) and sc.shape == (64, 4)
    assert torch.equal(M.deq_rows(q4, sc).half(), x)


def test_vt_key_order_and_round_trip():
    order = M.vt_key_order()
    assert sorted(order.flatten().tolist()) == list(range(64))
    assert ((order >> 2) & 1 == torch.arange(2)[:, None]).all()   # half h = keys with bit 2 == h
    g = torch.Generator().manual_seed(1)
    BH, Sk, D = 2, 128, 64
    codes = torch.randint(0, 16, (BH, Sk, D), generator=g)
    f = torch.randint(-4, 4, (BH, Sk // 64, D), generator=g).double()
    v = M.decode(codes).reshape(BH, Sk // 64, 64, D)
    v[:, :, 0] = 6.0                      # key 0 sits in half 0, key 4 in half 1
    v[:, :, 4] = -6.0
    v = (v * torch.pow(2.0, f)[:, :, None, :]).reshape(BH, Sk, D).half()
    vt, vs = M.quant_vt(v)
    assert vt.shape == (BH, 2, D, 32) and vs.shape == (BH, 2, D, 2)
    assert torch.equal(M.deq_vt(vt, vs).half(), v)


def test_fwd_uniform_keys_is_mean_of_values():
    """k = 0: every score is 0, P = 1 quantises exactly, so O = the mean of the dequantised V."""
    g = torch.Generator().manual_seed(2)
    q = torch.randn((1, 2, 32, 128), generator=g).half()
    k = torch.zeros((1, 2, 128, 128)).half()
    v = torch.randn((1, 2, 128, 128), generator=g).half()
    O, lse, ops = M.mxfp4_fwd(q, k, v)
    vd = M.deq_vt(ops[4], ops[5]).float()
    assert torch.allclose(O.float(), vd.mean(1, keepdim=True).view(1, 2, 1, 128).expand_as(O), atol=1e-3)
    assert torch.allclose(lse, torch.full_like(lse, 7.0))


def test_fwd_accuracy_vs_fp32_attention():
    """Accuracy bound of the FP4 definition on Gaussian data (measured cos ~0.97, relL2 ~0.24)."""
    g = torch.Generator().manual_seed(3)
    q = torch.randn((1, 4, 64, 128), generator=g).half()
    k = torch.randn((1, 2, 256, 128), generator=g).half()
    v = torch.randn((1, 2, 256, 128), generator=g).half()
    O, lse, _ = M.mxfp4_fwd(q, k, v)
    kk, vv = k.repeat_interleave(2, 1), v.repeat_interleave(2, 1)
    ref = R.baseline_pytorch_attention(q.float(), kk.float(), vv.float(), 128, False)
    cos = torch.nn.functional.cosine_similarity(O.float().flatten(), ref.flatten(), 0).item()
    assert cos >= 0.95, cos
    s = (q.float() @ kk.float().transpose(-1, -2)) * R.qk_scale(128)
    lref = torch.logsumexp(s * 0.6931471805599453, -1) / 0.6931471805599453
    assert (lse.view(1, 4, 64) - lref).abs().max().item() <= 0.3
