"""torch.library operators (quantizedattention_amd/ops.py): registration and fake-tensor
shape propagation on CPU; on the GPU, the operators equal the drop-in functions and trace into one
graph node each under torch.compile(fullgraph=True)."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import quantizedattention_amd.ops  # noqa: F401  (registers torch.ops.qattn.*)


def test_ops_registered():
    for name in ("int8_quant", "int8_fwd", "int8_bwd", "bf16_fwd", "bf16_bwd", "jvp_fwd", "mxfp4_fwd"):
        assert hasattr(torch.ops.qattn, name), name


def test_fake_shapes():
    with FakeTensorMode() as mode:
        q = torch.empty((2, 8, 256, 128), dtype=torch.float16, device="cuda")
        k = torch.empty((2, 2, 512, 128), dtype=torch.float16, device="cuda")
        O, lse, qi, ki, vi, sq, sk, sv = torch.ops.qattn.int8_fwd(q, k, k, True, False)
        assert O.shape == q.shape and O.dtype == torch.float16
        assert lse.shape == (2 * 8 * 256,) and qi.shape == (2 * 8 * 256, 128) and qi.dtype == torch.int8
        assert ki.shape == (2 * 2 * 512, 128) and sk.shape == (2 * 2 * 512 // 32,)
        dq, dk, dv = torch.ops.qattn.int8_bwd(O, qi, sq, ki, sk, vi, sv, O, lse, False, 2)
        assert dq.shape == q.shape and dk.shape == k.shape and dv.dtype == torch.float16
        Ob, lseb = torch.ops.qattn.bf16_fwd(q, k, k.bfloat16(), True)
        assert Ob.dtype == torch.float32 and lseb.shape == (16, 256)
        gq, gk, gv = torch.ops.qattn.bf16_bwd(q, k, k, Ob, lseb, True, Ob)
        assert gk.shape == k.shape and gq.dtype == torch.float32
        Oj, tOj, lj = torch.ops.qattn.jvp_fwd(q, k, k, q, k, k)
        assert tOj.shape == q.shape and lj.shape == (16, 256)
        assert torch.ops.qattn.mxfp4_fwd(q, k, k).shape == q.shape
        idx, sc = torch.ops.qattn.int8_quant(k, 32)
        assert idx.shape == k.shape and idx.dtype == torch.int8 and sc.shape == (2, 2, 16)
    assert mode is not None


@pytest.mark.gpu
def test_ops_match_dropins_and_compile(lib):
    from quantizedattention_amd.attention_bf16 import helion_atten_bf16_fwd_training
    from quantizedattention_amd.attention_int8 import helion_atten_int8_hl_dot_fwd
    g = torch.Generator(device="cuda").manual_seed(3)
    q, k, v = (torch.randn((1, 4, 256, 128), device="cuda", generator=g).half() for _ in range(3))
    out = torch.ops.qattn.int8_fwd(q, k, v, False, False)
    ref = helion_atten_int8_hl_dot_fwd(q, k, v)
    assert torch.equal(out[0], ref[0]) and torch.equal(out[3], ref[3].t())
    Ob, lb = torch.ops.qattn.bf16_fwd(q, k, v.bfloat16(), False)
    Rb, rl = helion_atten_bf16_fwd_training(q, k, v.bfloat16(), False)
    assert torch.equal(Ob, Rb) and torch.equal(lb, rl)

    def f(q, k, v):
        O, lse, *_ = torch.ops.qattn.int8_fwd(q, k, v, True, False)
        return O.float() * 2.0

    cf = torch.compile(f, backend="eager", fullgraph=True)
    assert torch.equal(cf(q, k, v), f(q, k, v))


@pytest.mark.gpu
def test_ops_autograd_matches_dropins(lib):
    """Autograd through torch.ops.qattn.int8_fwd / bf16_fwd equals the drop-in autograd Functions
    (int8: bit-identical -- the op rebuilds the bf16 images the drop-in forward writes)."""
    from quantizedattention_amd.attention_bf16 import flash_atten_2_bf16
    from quantizedattention_amd.attention_int8 import sage_attention_3_int8
    g = torch.Generator(device="cuda").manual_seed(5)
    q, k, v = (torch.randn((1, 4, 256, 128), device="cuda", generator=g).half() for _ in range(3))
    dO = torch.randn((1, 4, 256, 128), device="cuda", generator=g).half()
    a = [t.clone().requires_grad_(True) for t in (q, k, v)]
    b = [t.clone().requires_grad_(True) for t in (q, k, v)]
    torch.ops.qattn.int8_fwd(*a, True, False)[0].backward(dO)
    sage_attention_3_int8(*b).backward(dO)
    for x, y in zip(a, b):
        assert torch.equal(x.grad, y.grad)
    vb = v.bfloat16()
    a = [t.clone().requires_grad_(True) for t in (q, k, vb)]
    b = [t.clone().requires_grad_(True) for t in (q, k, vb)]
    torch.ops.qattn.bf16_fwd(*a, False)[0].backward(dO.float())
    flash_atten_2_bf16(*b, False).backward(dO.float())
    for x, y in zip(a, b):
        assert torch.equal(x.grad, y.grad)


@pytest.mark.gpu
def test_int8_quant_op_bit_exact(lib):
    """qattn::int8_quant equals the oracle's restatement of the reference quantiser bit for bit
    (including an all-zero block)."""
    from oracle import restate as R
    g = torch.Generator().manual_seed(3)
    x = (torch.randn((2, 3, 128, 128), generator=g) * 4).half()
    x[0, 1, 32:64] = 0
    idx, sc = torch.ops.qattn.int8_quant(x.cuda(), 32)
    ridx, rsc = R.quant_blocks(x)
    assert torch.equal(idx.cpu(), ridx) and torch.equal(sc.cpu(), rsc)
    with pytest.raises(ValueError):
        torch.ops.qattn.int8_quant(x.cuda(), 64)


def test_ops_are_cpp():
    """The qattn:: schemas and their CUDA kernels come from libqattn_torch.so (TORCH_LIBRARY in
    csrc/torch/qattn_ops.cpp), not from Python custom ops; no CPU kernel is registered."""
    from quantizedattention_amd import _lib
    assert (_lib._PKG / "libqattn_torch.so").exists()
    for name in ("int8_quant", "int8_fwd", "int8_bwd", "bf16_fwd", "bf16_bwd", "jvp_fwd", "mxfp4_fwd"):
        op = getattr(torch.ops.qattn, name).default
        assert torch._C._dispatch_has_kernel_for_dispatch_key(op.name(), "CUDA"), name
        assert not torch._C._dispatch_has_kernel_for_dispatch_key(op.name(), "CPU"), name
    with pytest.raises(NotImplementedError):
        torch.ops.qattn.int8_quant(torch.zeros((1, 1, 32, 64), dtype=torch.float16), 32)
    deps = open("/proc/self/maps").read()
    assert "libqattn_torch.so" in deps and "libqattn.so" in deps
