#!/bin/bash
# Stall-analysis PMC passes over tools/kernel_runner.py <kernels> (dev tool; GPU box, repo root):
#   tools/pmc_deep.sh <tag> [kernels]   -> gpurun_out/pmc_<tag>/p{1,2,3}/
set -e
TAG=$1; K=${2:-int8_all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P3="SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_WAVES SQ_INSTS_VMEM"
i=1
for P in "$P1" "$P2" "$P3"; do
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/tools/kernel_runner.py $K 2 > /dev/null 2>&1
  echo "pass $i done"
  i=$((i+1))
done
