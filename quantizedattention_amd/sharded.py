"""Head x batch sharding of the attention ops across the GPUs of one node.

Attention is independent per (batch, head), so each rank computes its own slice with no exchange
inside the operator.  The one collective is an all-gather of O (RCCL over xGMI,
``torch.distributed`` backend ``nccl``) for callers that want the full output replicated; it can run
asynchronously (``async_op=True``) so that it overlaps the backward kernels of the same step.

Partitioning: along B when B % world == 0 (each rank owns whole batches, its O shard
[B/world, H, S, D] is contiguous), otherwise along the flattened B*H axis (requires
(B*H) % world == 0).  Either way shards are contiguous in the flattened [B*H, S, D] view, so the
gather is a single ``all_gather_into_tensor`` with no reordering.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class Shard:
    world: int
    rank: int
    bh0: int      # first flattened (b*H + h) row owned by this rank
    bh1: int      # one past the last

    @property
    def n(self) -> int:
        return self.bh1 - self.bh0


def shard_for(batch: int, heads: int, world: int, rank: int) -> Shard:
    """Contiguous (b, h) range of ``rank`` (split along B when possible, else along B*H)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    bh = batch * heads
    if batch % world == 0:
        per = batch // world
        return Shard(world, rank, rank * per * heads, (rank + 1) * per * heads)
    if bh % world == 0:
        per = bh // world
        return Shard(world, rank, rank * per, (rank + 1) * per)
    raise ValueError(f"cannot shard B*H = {bh} evenly over {world} ranks")


def local_slice(x: torch.Tensor, shard: Shard) -> torch.Tensor:
    """The [n_local_bh, S, D] slice of a full [B, H, S, D] tensor (a view when contiguous)."""
    B, H, S, D = x.shape
    return x.reshape(B * H, S, D)[shard.bh0:shard.bh1]


def as_bhsd(x_flat: torch.Tensor, batch: int, heads: int) -> torch.Tensor:
    return x_flat.reshape(batch, heads, *x_flat.shape[-2:])


def all_gather_bh(local: torch.Tensor, out: torch.Tensor | None = None, group=None,
                  async_op: bool = False):
    """All-gather equal-size [n, ...] shards along dim 0 into [world * n, ...].

    Returns (out, work); ``work`` is None unless ``async_op``.
    """
    world = dist.get_world_size(group)
    local = local.contiguous()
    if out is None:
        out = torch.empty((world * local.shape[0], *local.shape[1:]), dtype=local.dtype,
                          device=local.device)
    work = dist.all_gather_into_tensor(out, local, group=group, async_op=async_op)
    return out, work


def kv_shard(shard: Shard, heads: int, kv_heads: int) -> Shard:
    """The key/value heads a query-head shard reads under grouped-query attention (query head h of
    batch b reads key/value head h // G, G = heads / kv_heads): in the flattened views the key/value
    row of query row i is i // G, so the shard's key/value range is [bh0 / G, bh1 / G).  Raises unless
    the shard holds whole groups (both bounds multiples of G)."""
    if heads % kv_heads:
        raise ValueError(f"query heads {heads} are not a multiple of key/value heads {kv_heads}")
    G = heads // kv_heads
    if shard.bh0 % G or shard.bh1 % G:
        raise ValueError(f"shard [{shard.bh0}, {shard.bh1}) splits a group of {G} query heads that "
                         "share a key/value head")
    return Shard(shard.world, shard.rank, shard.bh0 // G, shard.bh1 // G)


def sharded_forward(fn, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, *, group=None,
                    gather: bool = True):
    """Run ``fn(q_loc, k_loc, v_loc) -> O_loc (or a tuple whose [0] is O)`` on this rank's slice of
    full [B, H, S, D] inputs and (optionally) all-gather O to every rank.  k and v may have fewer
    heads (grouped-query attention): each rank gets the key/value heads its query heads read
    (:func:`kv_shard`), as [1, n / G, Sk, D] (n key/value rows, one per query head, when its range
    splits a group).

    A shard that splits a group of query heads sharing a key/value head (uneven splits) runs with
    one key/value copy per local query head instead.

    Returns (O_full or O_local as [B', H', S, D], the raw local result of ``fn``).
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    B, H, S, D = q.shape
    if k.shape[0] != B or v.shape[:2] != k.shape[:2]:
        raise ValueError("sharded_forward: k and v need q's batch and one head count")
    sh = shard_for(B, H, world, rank)
    ql = local_slice(q, sh).unsqueeze(0)
    Hkv = k.shape[1]
    if H % Hkv:
        raise ValueError(f"query heads {H} are not a multiple of key/value heads {Hkv}")
    G = H // Hkv
    if sh.bh0 % G == 0 and sh.bh1 % G == 0:
        kvs = kv_shard(sh, H, Hkv)
        kl, vl = (local_slice(t, kvs).unsqueeze(0) for t in (k, v))
    else:
        # the shard splits a group of query heads that share a key/value head: give every local
        # query head its own copy of the key/value head it reads (group 1 locally; same results)
        rows = torch.arange(sh.bh0, sh.bh1, device=k.device) // G
        kl, vl = (t.reshape(B * Hkv, *t.shape[2:]).index_select(0, rows).unsqueeze(0) for t in (k, v))
    res = fn(ql.contiguous(), kl.contiguous(), vl.contiguous())
    O_loc = res[0] if isinstance(res, tuple) else res
    if world == 1:   # the one shard is the whole problem: hand it back in the caller's layout
        return as_bhsd(O_loc.reshape(sh.n, S, -1), B, H), res
    if not gather:
        return O_loc, res
    full, _ = all_gather_bh(O_loc.reshape(sh.n, S, -1), group=group)
    return as_bhsd(full, B, H), res
