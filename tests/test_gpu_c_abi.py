"""The drop-in boundary without Python: tests/c_abi/int8_step (a plain C++ host of include/qattn.h,
linked to libqattn.so, no torch) runs the int8 training step -- k-smoothing, the quantisers with
the bf16 images, the int8 forward (P.V on the int8 MFMA), the backward prologue and the dS-record
backward -- and every output must equal, bit for bit, what the Python drop-in
(sage_attention_3_int8 forward + backward, attention_int8.py) computes on the same inputs.  This is
the call sequence INTEGRATION.md gives a non-Python binding."""
import os
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c_abi", "int8_step")


@pytest.mark.parametrize("shape", [(2, 4, 512, 128), (1, 3, 256, 64)])
def test_c_host_matches_the_python_drop_in(shape, tmp_path):
    assert os.path.exists(BIN), "tests/c_abi/int8_step not built (run __graft_entry__.build())"
    from quantizedattention_amd import attention_int8 as A
    B, H, S, D = shape
    g = torch.Generator().manual_seed(7)
    ins = {"q": torch.randn(shape, generator=g).half(), "k": torch.randn(shape, generator=g).half(),
           "v": torch.randn(shape, generator=g).half(),
           "dO": (torch.randn(shape, generator=g) * 0.1).half()}
    for name, t in ins.items():
        t.numpy().tofile(tmp_path / f"{name}.f16")
    r = subprocess.run([BIN, str(B), str(H), str(S), str(D), str(tmp_path)], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    q, k, v, dO = (ins[n].cuda() for n in ("q", "k", "v", "dO"))
    # the Python drop-in: autograd function of attention_int8.py
    qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
    out = A.sage_attention_3_int8(qq, kk, vv)
    out.backward(dO)
    O, lse, *_ = A._int8_forward(q, k, v, smooth=True, images=True)
    torch.cuda.synchronize()

    def load(name, n):
        return torch.from_numpy(np.fromfile(tmp_path / f"{name}.f16", dtype=np.float16, count=n))

    n = B * H * S * D
    want = {"O": out, "lse": lse, "dq": qq.grad, "dk": kk.grad, "dv": vv.grad}
    assert torch.equal(O.cpu(), out.detach().cpu())
    for name, t in want.items():
        got = load(name, t.numel()).view(t.shape)
        assert torch.equal(got, t.detach().cpu()), f"{name} differs between the C host and Python"
    assert want["dq"].numel() == n and torch.isfinite(want["dq"].float()).all()
