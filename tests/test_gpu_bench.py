"""bench.py's output contract (one JSON line on rank 0) on a small shape, run as the driver runs it:
a child process on the GPU.  The numbers themselves are measured elsewhere (profiles/)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--shape",
                        "1,4,1024,128", "--cpu-seconds", "1"], cwd=ROOT, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["value"] > 0
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and "workload" in d["config"]
    assert "(1,4,1024,128)" in d["config"]["workload"]
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["unit"] in ("GB/s", "TFLOP/s")
    assert 0 < rf["frac"] < 1 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] in ("port", "reference") and cb["cores"] >= 1
    assert cb["logical_cpus"] >= cb["cores"] and "cpu_model" in cb
