"""The int8 O bars against an oracle whose exp2 is one ulp low.

The oracle (oracle/restate.py `_exp2`) pins exp2 to the correctly rounded value, and so do the
kernels (the exp2 correction table).  The reference's torch.exp2 is whatever its
platform computes, within an ulp, and one ulp of it moves the reference's own O by up to 6.3e-3 on
peaked rows (tests/test_oracle_sensitivity.py).  So the 1e-2 bar of the parity tests assumes a
correctly rounded exp2 on the reference's side.  This test drops that assumption: against the oracle
with exp2 one ulp down wherever it is inexact (`exp2_down`), the kernel must stay within
  * the north star's 1e-2 on random inputs (where one ulp moves O by < 2e-3), and
  * the round-4 bar 3e-2 on the peaked rows of tests/test_gpu_edge.py.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _exp2_down(orig):
    def f(x):
        y = orig(x)
        return torch.where(y == torch.round(y), y, torch.nextafter(y, torch.zeros_like(y)))
    return f


@pytest.mark.parametrize("kind", ["random", "peaked"])
def test_int8_O_against_exp2_one_ulp_down(lib, monkeypatch, kind):
    from oracle import restate as R
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    g = torch.Generator().manual_seed(71)
    S, D = 256, 128
    if kind == "random":
        q, k, v = (torch.randn((1, 4, S, D), generator=g).half() for _ in range(3))
        bar = 1e-2
    else:
        ramp = (1.0 + torch.arange(S, dtype=torch.float32) / 24.0).view(1, 1, S, 1)
        k = (torch.randn((1, 2, S, D), generator=g) * ramp).half()
        q = k.clone()
        v = torch.randn((1, 2, S, D), generator=g).half()
        bar = 3e-2
    out = helion_atten_int8_hl_dot_fwd(q.cuda(), k.cuda(), v.cuda())
    O = out[0].float().cpu()
    exact = R.int8_fwd(q, k, v)[0].float()
    monkeypatch.setattr(R, "_exp2", _exp2_down(R._exp2))
    down = R.int8_fwd(q, k, v)[0].float()
    d_exact = (O - exact).abs().max().item()
    d_down = (O - down).abs().max().item()
    moved = (down - exact).abs().max().item()
    print(f"{kind}: |O - O_ref| {d_exact:.2e}, |O - O_ref(exp2 - 1 ulp)| {d_down:.2e}, "
          f"oracle moved {moved:.2e}")
    assert d_exact <= 1e-2
    assert d_down <= bar
