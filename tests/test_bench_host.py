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


def test_chunk_heads_match_the_step():
    """bench.py times the record backward as the step launches it: chunks of >= 512 dK+dV
    workgroups (attention_int8._ws_chunk), 32 heads at config 3 -> 4 launches per step."""
    assert bench.ws_chunk_heads(128, 4096) == 32
    assert bench.ws_chunk_heads(4, 256) == 4        # small problems: one launch over all heads


def test_profile_tools_tell_grids_apart(tmp_path):
    """tools/profile_summary.key_of separates the chunk-sized and one-pass launches of the same
    kernel by their grids, and tools/trace_summary.py groups a kernel trace per (kernel, grid)."""
    import csv
    import subprocess
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from profile_summary import key_of, workgroups
    name = "void qattn::int8_bwd_kernel<128, 3, false, true>(signed char const*)"
    assert key_of(name, 512) == "int8_bwd_dkdv_kernel<dK+dV, dS out>"
    assert key_of(name, 2048) == "int8_bwd_dkdv_kernel<dK+dV, dS out, one pass>"
    fwd = "void qattn::int8_attn_fwd_kernel<128, false, false, true, false, true>(signed char const*)"
    assert key_of(fwd, 4096) == "int8_attn_fwd_kernel"
    fwd = "void qattn::int8_attn_fwd_kernel<128, false, false, false, false, false>(signed char const*)"
    assert key_of(fwd, 4096) == "int8_attn_fwd_kernel<q_i8 in>"
    assert workgroups({"Grid_Size_X": "262144", "Workgroup_Size_X": "512"}) == 512
    d = tmp_path / "trace"
    d.mkdir()
    cols = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X",
            "LDS_Block_Size"]
    rows = [(name, 0, 500, 262144, 512, 1024), (name, 1000, 1510, 262144, 512, 1024),
            (name, 2000, 4000, 1048576, 512, 1024)]
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        w.writerows(rows)
    out = tmp_path / "shapes.csv"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_summary.py"), str(d), str(out)],
                   check=True, capture_output=True)
    got = {r["bench_key"]: r for r in csv.DictReader(open(out))}
    assert got["int8_bwd_dkdv_kernel<dK+dV, dS out>"]["Calls"] == "2"
    assert got["int8_bwd_dkdv_kernel<dK+dV, dS out>"]["AverageNs"] == "505"
    assert got["int8_bwd_dkdv_kernel<dK+dV, dS out, one pass>"]["AverageNs"] == "2000"
