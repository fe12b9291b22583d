"""The multi-GPU path on a GPU at world size 1: RCCL (backend "nccl") initialised in a
clean child process before any other GPU work, ``sharded_forward`` over the HIP int8 op, and the
bench's step pattern (async all-gather of O on a side stream beside the backward) -- each compared
bit for bit with the unsharded call.  (8-rank runs are the driver's; the partition itself is covered
at world size 2 on gloo in tests/test_sharded.py.)"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import os, sys, torch, torch.distributed as dist
    sys.path.insert(0, {root!r})
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    from quantizedattention_amd.sharded import sharded_forward, all_gather_bh
    from quantizedattention_amd.attention_int8 import (sage_attention_3_int8, _int8_forward,
                                                       _int8_backward)
    g = torch.Generator(device="cuda").manual_seed(11)
    B, H, Hkv, S, D = 2, 4, 2, 256, 128
    q = torch.randn((B, H, S, D), device="cuda", generator=g).half()
    k, v = (torch.randn((B, Hkv, S, D), device="cuda", generator=g).half() for _ in range(2))
    O_sh, _ = sharded_forward(lambda a, b, c: sage_attention_3_int8(a, b, c), q, k, v)
    O_ref = sage_attention_3_int8(q, k, v)
    assert torch.equal(O_sh, O_ref), "sharded_forward differs from the unsharded call"
    # the all-gather itself (world 1: a copy through RCCL)
    full, work = all_gather_bh(O_ref.reshape(B * H, S, D), async_op=True)
    work.wait()
    assert torch.equal(full.view(B, H, S, D), O_ref)
    # bench.py's step: the gather of O on a side stream, the backward on the compute stream
    dO = (torch.randn((B, H, S, D), device="cuda", generator=g) * 1e-3).half()
    O, lse, qi, kiT, vi, sq, sk, sv, km, qb, kb = _int8_forward(q, k, v, smooth=True, images=True)
    O_full = torch.empty((B * H, S, D), dtype=torch.float16, device="cuda")
    comm = torch.cuda.Stream(device=dev)
    comm.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(comm):
        work = dist.all_gather_into_tensor(O_full, O.view(B * H, S, D), async_op=True)
    grads = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, kv_heads=Hkv)
    work.wait()
    torch.cuda.current_stream().wait_stream(comm)
    torch.cuda.synchronize()
    assert torch.equal(O_full.view(B, H, S, D), O)
    ref = _int8_backward(dO, qi, sq, kiT, sk, vi, sv, O, lse, qb, kb, kv_heads=Hkv)
    for a, b in zip(grads, ref):
        assert torch.equal(a, b), "backward beside the gather differs"
    dist.destroy_process_group()
    print("SHARDED_OK")
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_nccl_world1_bit_identical():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               LOCAL_RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "SHARDED_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
