"""The HIP kernels against the numbers the reference itself publishes.

The reference asserts nothing; the only numbers it holds for this path are two accuracy
statistics in its test drivers, both at (B,H,S,D) = (8,35,1024,64):

* attention_jvp.py:305-317 — fp32 JVP vs torch.func.jvp: 0 elements of O or tO with |diff| > 1e-2,
  MSE(O) = 6.6253e-09, MSE(tO) = 1.2681e-07 (tangents all ones, jvp:242-245).  The HIP fp32 (X3)
  JVP is checked against exactly these bars, on the published shape.
* attention_bf16.py:563 — bf16 forward, causal: 915 of 18,350,080 elements with |O - O_fp32| > 1e-2.
  That count depends on the k-tile the literal beta rule is evaluated at (the reference's
  forward has no pinned config, so its run used Helion's default tile).  The oracle brackets the
  published count between k-tiles 256 and 64 (tests/test_oracle.py::test_pin_bf16_published_error_rate);
  the HIP kernel evaluates the rule per 16 keys (the tuned config, bf16:736), so here its count on
  the published shape is tied to the oracle's count at the same k-tile (within 10 %), and the count
  of the oracle at the bracketing tiles to the published one.
"""
import pytest
import torch

from oracle import restate as R

pytestmark = pytest.mark.gpu

PUBLISHED_BF16 = 915 / 18350080


def test_pin_jvp_fp32_published_accuracy(lib):
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn((8, 35, 1024, 64), device="cuda", generator=g) for _ in range(3))
    t = torch.ones_like(q)
    O, tO, _ = helion_attention_jvp_forward_fp32(q, k, v, t, t, t)
    Ot, tOt = R.jvp_truth(q, k, v, t, t, t)   # fp32 torch.func.jvp on the GPU, as jvp:254-258
    torch.cuda.synchronize()
    assert int((~torch.isclose(Ot, O, atol=1e-2, rtol=0)).sum()) == 0
    assert int((~torch.isclose(tOt, tO, atol=1e-2, rtol=0)).sum()) == 0
    assert torch.nn.functional.mse_loss(Ot, O).item() <= 6.6253e-09
    assert torch.nn.functional.mse_loss(tOt, tO).item() <= 1.2681e-07


def test_pin_bf16_published_error_rate(lib):
    from quantizedattention_amd.attention_bf16 import KT, helion_atten_bf16_fwd_training
    g = torch.Generator().manual_seed(0)
    q, k, v = (torch.randn((2, 35, 1024, 64), generator=g) for _ in range(3))
    truth = R.baseline_pytorch_attention(q.cuda(), k.cuda(), v.cuda(), 64, True)
    O, _ = helion_atten_bf16_fwd_training(q.half().cuda(), k.half().cuda(), v.bfloat16().cuda(), True)
    n_hip = int((~torch.isclose(truth, O, atol=1e-2, rtol=0)).sum())
    truth = truth.cpu()
    rates = {}
    for kt in sorted({KT, 64, 256}):
        O_ref, _ = R.bf16_fwd(q.half(), k.half(), v.bfloat16(), True, kt=kt)
        rates[kt] = int((~torch.isclose(truth, O_ref, atol=1e-2, rtol=0)).sum())
    assert abs(n_hip - rates[KT]) <= 0.1 * rates[KT] + 10, (n_hip, rates)
    n = O.numel()
    assert rates[256] / n <= PUBLISHED_BF16 <= rates[64] / n, rates
