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
