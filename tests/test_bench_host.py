"""Host logic of bench.py (no GPU): the --gpus N launcher, the config-4 sharding of the global
problem, the CPU-baseline core accounting and the traffic source hash."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_gpus_n_without_torchrun_spawns_ranks(monkeypatch):
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7
    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "5"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "5"]


def test_world_size_mismatch_fails_fast(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_config4_shards_cover_the_global_problem(world):
    """Rank r's heads are rows [r*256/N, (r+1)*256/N) of the global (8*32) heads: together exactly
    the global problem, each rank's slice contiguous."""
    from quantizedattention_amd.sharded import shard_for
    covered = []
    for r in range(world):
        sh = bench.shard_for(8, 32, world, r)
        assert sh == shard_for(8, 32, world, r) and sh.n == 256 // world
        covered += list(range(sh.bh0, sh.bh1))
    assert covered == list(range(256))


def test_cpu_info_and_threads():
    info = bench.cpu_info()
    assert info["logical_cpus"] == os.cpu_count() and info["affinity_cpus"] >= 1
    assert info["physical_cores"] is None or 1 <= info["physical_cores"] <= info["logical_cpus"]


def test_source_hash_tracks_the_kernel_sources():
    h = bench.source_hash()
    assert len(h) == 64 and h == bench.source_hash()
