#!/bin/bash
# Round profile (runs on the GPU box from the repo root):  tools/profile_round.sh <tag>
#   1. rocprofv3 --kernel-trace --stats of the default bench command (N=1)  -> per-kernel durations
#   2. separate --pmc passes FETCH_SIZE / WRITE_SIZE over tools/kernel_runner.py int8_all
#      (MI355X_MICROARCH.md "HBM": one TCC counter group per pass; FETCH_SIZE x2 on gfx950)
# Summaries land in gpurun_out/prof_<tag>/ ; tools/profile_summary.py turns them into profiles/.
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
echo "trace done"
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "fetch done"
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "write done"
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv \
  -d $OUT/mfma -o run -- python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "mfma done"
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 \
  --output-format csv -d $OUT/mops -o run -- python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "mops done"
