#!/bin/bash
# Round profile (runs on the GPU box from the repo root):  tools/profile_round.sh <tag>
# One run on the current sources, in this order, so that the bench line carries roofline.traffic:
#   1. separate rocprofv3 --pmc passes over tools/kernel_runner.py int8_all (MI355X_MICROARCH.md
#      "HBM": one TCC counter group per pass; FETCH_SIZE x2 on gfx950), the chunk-sized launches the
#      step runs and the one-pass launches told apart by their grids
#   2. tools/profile_summary.py -> <out>/profiles/<tag>_pmc.json and traffic_latest.json (also copied
#      to profiles/ here, where bench.py reads it)
#   3. rocprofv3 --kernel-trace --stats of the bench command without the other-config leg (every
#      launch config 3), and tools/trace_summary.py: per (kernel, grid, LDS) rows
#      (<tag>_kernel_shapes.csv) beside rocprof's per-name --stats table
#   4. the plain `python bench.py` line (roofline with traffic, cpu_baseline)
# Everything lands in gpurun_out/prof_<tag>/ (merged back by gpurun); copy profiles/ from there.
set -e
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT/profiles
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "fetch done"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "write done"
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --output-format csv \
  -d $OUT/mfma -o run -- python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "mfma done"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 \
  --output-format csv -d $OUT/mops -o run -- python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "mops done"
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/valu -o run -- python3 $R/tools/kernel_runner.py int8_all 2 > /dev/null 2>&1
echo "valu done"
cd $R
python3 tools/profile_summary.py $OUT $TAG $OUT/profiles > $OUT/pmc_summary.txt
cp $OUT/profiles/traffic_latest.json profiles/traffic_latest.json
echo "pmc summary done"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-configs > $OUT/bench_traced.json 2> $OUT/bench_traced.err
cd $R
cp $(find $OUT/bench -name '*kernel_stats.csv' | head -n 1) $OUT/profiles/${TAG}_kernel_stats.csv
python3 tools/trace_summary.py $OUT/bench $OUT/profiles/${TAG}_kernel_shapes.csv
echo "trace done"
timeout -k 10 400 python3 bench.py > $OUT/profiles/${TAG}_bench.json 2> $OUT/bench.err
tail -c 400 $OUT/profiles/${TAG}_bench.json
