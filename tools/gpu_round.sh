#!/bin/bash
# One GPU round (runs on the GPU box from the repo root):  tools/gpu_round.sh <tag>
#   GPU test suite, smoke(), then tools/profile_round.sh <tag> (PMC passes, traced bench, plain bench).
# Stops at the first failing step (no GPU step runs after a failure or a time-out).
set -o pipefail
TAG=${1:?tag}
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/prof_$TAG/profiles
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/prof_$TAG/profiles/${TAG}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/prof_$TAG/profiles/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/prof_$TAG/profiles/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/prof_$TAG/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/prof_$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/prof_$TAG/smoke.log
bash tools/profile_round.sh $TAG
