#!/bin/bash
# usage: tools/pmc.sh <kernel_runner name> <outdir>   (runs on the GPU box; separate --pmc passes,
# each under its own hard time limit: a pass that over-asks a counter block hangs after printing
# "error code 38" -- MI355X_MICROARCH.md "rocprofv3 PMC slots")
set -e
NAME=$1; OUT=$(realpath -m $2)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() { local tag=$1; shift; timeout -s KILL 90 rocprofv3 "$@" --output-format csv -d $OUT/$tag -o run -- python3 $R/tools/kernel_runner.py $NAME 2 > /dev/null; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/kernel_runner.py $NAME 5 > /dev/null
run p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES
run p2 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run p3 --pmc FETCH_SIZE
run p4 --pmc WRITE_SIZE
run p5 --pmc TCC_HIT_sum TCC_MISS_sum
run p6 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES
echo pmc done
