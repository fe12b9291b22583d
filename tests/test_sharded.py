"""Head x batch sharding on CPU: partition math and the world-size-2 gloo all-gather.

The GPU path is the same code over RCCL (backend "nccl"); here the per-rank attention is the
oracle's fp32 baseline so that the test needs no GPU.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from quantizedattention_amd.sharded import (Shard, all_gather_bh, kv_shard, local_slice, shard_for,
                                            sharded_forward)


@pytest.mark.parametrize("B,H,world", [(4, 32, 1), (4, 32, 2), (4, 32, 8), (8, 32, 8), (1, 16, 4),
                                       (2, 3, 3), (3, 4, 2)])
def test_shards_cover_exactly_once(B, H, world):
    seen = []
    for r in range(world):
        s = shard_for(B, H, world, r)
        assert s.n == B * H // world
        seen.extend(range(s.bh0, s.bh1))
    assert seen == list(range(B * H))


def test_shard_prefers_batch_split():
    s = shard_for(8, 32, 8, 3)
    assert (s.bh0, s.bh1) == (3 * 32, 4 * 32)


def test_shard_rejects_uneven():
    with pytest.raises(ValueError):
        shard_for(1, 3, 2, 0)
    with pytest.raises(ValueError):
        shard_for(2, 2, 2, 2)


@pytest.mark.parametrize("B,H,Hkv,world", [(2, 8, 2, 2), (1, 8, 4, 2), (4, 32, 8, 8), (8, 32, 1, 8)])
def test_kv_shard_pairs_query_heads_with_their_kv_heads(B, H, Hkv, world):
    """Grouped-query sharding: every query head of a rank finds its key/value head (h // G within its
    batch) inside the rank's key/value range."""
    G = H // Hkv
    for r in range(world):
        s = shard_for(B, H, world, r)
        kvs = kv_shard(s, H, Hkv)
        for i in range(s.bh0, s.bh1):
            b, h = divmod(i, H)
            kv_flat = b * Hkv + h // G
            assert kvs.bh0 <= kv_flat < kvs.bh1
            assert kv_flat - kvs.bh0 == (i - s.bh0) // G


def test_kv_shard_rejects_split_groups():
    assert kv_shard(shard_for(1, 6, 2, 0), 6, 2) == Shard(2, 0, 0, 1)   # 3 query heads = 1 group
    # H = 4, Hkv = 1 (G = 4) over 2 ranks of 2 query heads each: every rank splits the group
    with pytest.raises(ValueError, match="splits a group"):
        kv_shard(shard_for(1, 4, 2, 0), 4, 1)


def test_local_slice_is_view():
    x = torch.randn(2, 4, 8, 16)
    s = Shard(2, 1, 4, 8)
    v = local_slice(x, s)
    assert v.data_ptr() == x[1].data_ptr() and torch.equal(v, x[1])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, B, H, S, D, errq, Hkv=None):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle import restate as R
        g = torch.Generator().manual_seed(11)
        Hk = H if Hkv is None else Hkv
        q = torch.randn((B, H, S, D), generator=g)
        k, v = (torch.randn((B, Hk, S, D), generator=g) for _ in range(2))
        rep = lambda t: t.repeat_interleave(H // Hk, dim=1)  # noqa: E731
        full = R.baseline_pytorch_attention(q, rep(k), rep(v))

        def fn(ql, kl, vl):   # grouped-query attention on the local heads
            G = ql.shape[1] // kl.shape[1]
            return R.baseline_pytorch_attention(ql, kl.repeat_interleave(G, 1), vl.repeat_interleave(G, 1)), None

        O, res = sharded_forward(fn, q, k, v)
        assert O.shape == (B, H, S, D)
        assert torch.allclose(O, full, atol=1e-6), float((O - full).abs().max())
        loc = res[0]
        sh = shard_for(B, H, world, rank)
        assert loc.shape == (1, sh.n, S, D)
        # async gather completes to the same result
        out, work = all_gather_bh(loc.reshape(sh.n, S, D), async_op=True)
        work.wait()
        assert torch.allclose(out.reshape(B, H, S, D), full, atol=1e-6)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        errq.put(f"rank {rank}: {type(e).__name__}: {e}")
        raise


@pytest.mark.parametrize("B,H,Hkv", [(2, 4, None), (1, 6, None), (2, 8, 2), (1, 8, 2), (1, 4, 1), (1, 6, 3)])
def test_gloo_world2_sharded_forward(B, H, Hkv):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, H, 64, 32, errq, Hkv)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
