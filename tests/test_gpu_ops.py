"""The C++ operator layer (csrc/torch/qattn_ops.cpp) on the GPU: every qattn:: operator
is bit-identical to the Python drop-in that runs the same kernel sequence through ctypes, raises the
drop-ins' messages, and runs on the inputs' device and torch's current stream."""
import pytest
import torch

import quantizedattention_amd.ops  # noqa: F401  (loads libqattn_torch.so)

pytestmark = pytest.mark.gpu


def _rand(shape, g, dt=torch.float16, scale=1.0):
    return (torch.randn(shape, device="cuda", generator=g) * scale).to(dt)


@pytest.mark.parametrize("causal", [False, True])
def test_int8_ops_equal_dropins(lib, causal):
    from quantizedattention_amd.attention_int8 import _int8_backward, _int8_forward
    g = torch.Generator(device="cuda").manual_seed(11)
    q = _rand((2, 4, 256, 128), g)
    k, v = _rand((2, 2, 256, 128), g), _rand((2, 2, 256, 128), g)
    dO = _rand((2, 4, 256, 128), g, scale=1e-2)
    out = torch.ops.qattn.int8_fwd(q, k, v, True, causal)
    ref = _int8_forward(q, k, v, smooth=True, causal=causal)
    for i, (a, b) in enumerate(zip(out, ref[:8])):
        b = b.t() if i == 3 else b
        assert torch.equal(a, b.contiguous()), i
    O, lse, qi, ki, vi, sq, sk, sv = out
    got = torch.ops.qattn.int8_bwd(dO, qi, sq, ki, sk, vi, sv, O, lse, causal, 2)
    exp = _int8_backward(dO, qi, sq, ki.t(), sk, vi, sv, O, lse, causal=causal, kv_heads=2)
    for a, b in zip(got, exp):
        assert torch.equal(a, b)
    idx, sc = torch.ops.qattn.int8_quant(q, 32)
    assert torch.equal(idx.view(-1, 128), qi) and torch.equal(sc.reshape(-1), sq)


def test_int8_bwd_op_chunked_and_recompute_equal(lib, monkeypatch):
    """The operator's workspace policy (head chunks, one pass, recomputation) never changes the
    gradients."""
    g = torch.Generator(device="cuda").manual_seed(12)
    q, k, v = (_rand((1, 8, 512, 128), g) for _ in range(3))
    dO = _rand((1, 8, 512, 128), g, scale=1e-2)
    O, lse, qi, ki, vi, sq, sk, sv = torch.ops.qattn.int8_fwd(q, k, v, True, False)
    outs = []
    for env in ({"QATTN_BWD_WS_CHUNK": "3"}, {"QATTN_BWD_WS_CHUNK": "0"}, {"QATTN_BWD_WS_MAX": "0"}):
        for key in ("QATTN_BWD_WS_CHUNK", "QATTN_BWD_WS_MAX"):
            monkeypatch.delenv(key, raising=False)
        for key, val in env.items():
            monkeypatch.setenv(key, val)
        outs.append(torch.ops.qattn.int8_bwd(dO, qi, sq, ki, sk, vi, sv, O, lse, False, 8))
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("causal", [False, True])
def test_bf16_ops_equal_dropins(lib, causal):
    from quantizedattention_amd.attention_bf16 import (helion_atten_bf16_fwd_training,
                                                       helion_flash_atten_2_algo_4_bwd)
    g = torch.Generator(device="cuda").manual_seed(13)
    q, k = _rand((1, 4, 256, 128), g), _rand((1, 2, 256, 128), g)
    v = _rand((1, 2, 256, 128), g, torch.bfloat16)
    dO = _rand((1, 4, 256, 128), g, torch.float32)
    O, lse = torch.ops.qattn.bf16_fwd(q, k, v, causal)
    RO, rl = helion_atten_bf16_fwd_training(q, k, v, causal)
    assert torch.equal(O, RO) and torch.equal(lse, rl)
    got = torch.ops.qattn.bf16_bwd(q, k, v, O, lse, causal, dO)
    exp = helion_flash_atten_2_algo_4_bwd(q, k, v, O, lse, causal, dO)
    for a, b in zip(got, exp):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_jvp_op_equals_dropin(lib, dt):
    from quantizedattention_amd.attention_jvp import helion_attention_jvp_forward_fp32
    g = torch.Generator(device="cuda").manual_seed(14)
    x = [_rand((1, 2, 128, 64), g, dt) for _ in range(6)]
    got = torch.ops.qattn.jvp_fwd(*x)
    exp = helion_attention_jvp_forward_fp32(*x)
    for a, b in zip(got, exp):
        assert torch.equal(a, b)


def test_mxfp4_op_equals_dropin(lib):
    from quantizedattention_amd.attention_mxfp4 import sage_attention_3_fp4
    g = torch.Generator(device="cuda").manual_seed(15)
    q, k, v = (_rand((1, 2, 128, 128), g) for _ in range(3))
    assert torch.equal(torch.ops.qattn.mxfp4_fwd(q, k, v), sage_attention_3_fp4(q, k, v))


def test_op_errors_and_stream(lib):
    g = torch.Generator(device="cuda").manual_seed(16)
    q = _rand((1, 2, 64, 64), g)
    with pytest.raises(RuntimeError, match="k and v tokens are different"):
        torch.ops.qattn.int8_fwd(q, q, q[:, :, :32], False, False)
    with pytest.raises(RuntimeError, match="input k_tokens must match v_tokens"):
        torch.ops.qattn.bf16_fwd(q, q, q[:, :, :32].bfloat16(), False)
    with pytest.raises(RuntimeError, match="head_dim must be 64 or 128"):
        torch.ops.qattn.int8_fwd(q[..., :32], q[..., :32], q[..., :32], False, False)
    # enqueued on the current stream: a side stream's result equals the default stream's
    ref = torch.ops.qattn.int8_fwd(q, q, q, False, False)[0]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        out = torch.ops.qattn.int8_fwd(q, q, q, False, False)[0]
    torch.cuda.current_stream().wait_stream(s)
    assert torch.equal(out, ref)
