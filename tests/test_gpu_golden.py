"""GPU parity against the committed golden fixtures (tests/golden/oracle_small.pt, made by
tests/golden/gen_golden.py).  Same tolerances as the oracle-on-the-fly tests:
int8 indices/scales bit-exact, int8 O <= 1e-2, lse <= 2 fp16 ulp (+1e-3); int8 grads relL2 <= conftest.INT8_BWD_REL;
bf16 O <= 5e-3, bf16 grads relL2 <= 1e-2; jvp O/tO <= 1e-2 (inputs rounded to bf16)."""
from pathlib import Path

import pytest
import torch

from conftest import INT8_BWD_REL

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden" / "oracle_small.pt"


@pytest.fixture(scope="module")
def fx():
    return torch.load(GOLD, weights_only=True)


def _rel(a, b):
    return float((a.float().cpu() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("tag", ["i8a", "i8b"])
def test_int8_fwd_golden(lib, fx, tag):
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    q, k, v = (fx[f"{tag}.{n}"].cuda() for n in "qkv")
    out = helion_atten_int8_hl_dot_fwd(q, k, v)
    torch.cuda.synchronize()
    names = ("O", "lse", "q_i8", "k_i8T", "v_i8", "sq", "sk", "sv")
    got = {n: t.cpu() for n, t in zip(names, out[:8])}
    for n in ("q_i8", "k_i8T", "v_i8"):
        assert torch.equal(got[n], fx[f"{tag}.{n}"]), n
    for n in ("sq", "sk", "sv"):
        assert torch.equal(got[n].view(torch.int16), fx[f"{tag}.{n}"].view(torch.int16)), n
    assert (got["O"].float() - fx[f"{tag}.O"].float()).abs().max() <= 1e-2
    ref_lse = fx[f"{tag}.lse"].float()
    assert ((got["lse"].float() - ref_lse).abs() <= 2 * 2.0 ** -10 * ref_lse.abs() + 1e-3).all()
    assert out[8] == 32 and out[9] == 32


@pytest.mark.parametrize("tag", ["i8a", "i8b"])
def test_sage_fwd_bwd_golden(lib, fx, tag):
    from quantizedattention_amd.attention_int8 import SageAttention3_Int8_autograd_function as F
    q, k, v = (fx[f"{tag}.{n}"].cuda().requires_grad_(True) for n in "qkv")
    out = F.apply(q, k, v)
    assert (out[0].detach().float().cpu() - fx[f"{tag}.smooth.O"].float()).abs().max() <= 1e-2
    assert torch.equal(out[2].cpu().view(torch.int16), fx[f"{tag}.smooth.k_mean"].view(torch.int16))
    out[0].backward(fx[f"{tag}.dO"].cuda())
    for n, t in zip("qkv", (q, k, v)):
        rel = _rel(t.grad, fx[f"{tag}.smooth.d{n}"])
        print(f"RELL2 int8-bwd-vs-oracle d{n} {rel:.5f}")
        assert rel <= INT8_BWD_REL, (n, rel)


@pytest.mark.parametrize("causal", [0, 1])
def test_bf16_golden(lib, fx, causal):
    from quantizedattention_amd.attention_bf16 import (helion_atten_bf16_fwd_training,
                                                       helion_flash_atten_2_algo_4_bwd)
    q, k, v = fx["bf.q"].cuda(), fx["bf.k"].cuda(), fx["bf.v"].cuda()
    O, lse = helion_atten_bf16_fwd_training(q, k, v, bool(causal))
    assert (O.cpu() - fx[f"bf.c{causal}.O"]).abs().max() <= 5e-3
    assert (lse.cpu() - fx[f"bf.c{causal}.lse"]).abs().max() <= 5e-3
    dq, dk, dv = helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, bool(causal), fx["bf.dO"].cuda())
    for n, g in zip("qkv", (dq, dk, dv)):
        assert _rel(g, fx[f"bf.c{causal}.d{n}"]) <= 1e-2, n


def test_jvp_golden(lib, fx):
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    args = [fx[f"jvp.{n}"].cuda() for n in ("q", "k", "v", "tq", "tk", "tv")]
    O, tO, lse = helion_attention_jvp_forward_fp32(*args)
    assert (O.cpu() - fx["jvp.O"]).abs().max() <= 1e-2
    assert (tO.cpu() - fx["jvp.tO"]).abs().max() <= 3e-2
    assert (lse.cpu() - fx["jvp.lse"]).abs().max() <= 1e-2
