#!/bin/bash
# One GPU round (runs on the GPU box from the repo root):  tools/gpu_round.sh <tag>
#   GPU test suite, smoke(), the default bench line, then tools/profile_round.sh <tag>.
# Stops at the first failing step (no GPU step runs after a failure or a time-out).
set -o pipefail
TAG=${1:?tag}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 600 gpurun_out/${TAG}_bench.json
bash tools/profile_round.sh ${TAG}
