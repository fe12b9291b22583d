#!/bin/bash
# usage: tools/pmc.sh <kernel_runner name> <outdir>   (runs on the GPU box; separate --pmc passes)
set -e
NAME=$1; OUT=$(realpath -m $2)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/kernel_runner.py $NAME 5 > /dev/null
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -o run -- python3 $R/tools/kernel_runner.py $NAME 2 > /dev/null
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p2 -o run -- python3 $R/tools/kernel_runner.py $NAME 2 > /dev/null
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- python3 $R/tools/kernel_runner.py $NAME 2 > /dev/null
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o run -- python3 $R/tools/kernel_runner.py $NAME 2 > /dev/null
echo pmc done
