set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02a_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r02a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r02a_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a_smoke.log 2>&1 && tail -1 gpurun_out/r02a_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err && tail -c 600 gpurun_out/r02a_bench.json
bash tools/profile_round.sh r02a
