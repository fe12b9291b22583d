#!/bin/bash
# rocprofv3 kernel stats of `python3 <script> [args]` for the default library and _ab variants (dev tool)
#   tools/prof_ab.sh <script> "<args>" variant...   ("default" = the in-tree library)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
S=$1; A=$2; shift 2
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then unset QATTN_LIB; else export QATTN_LIB=$R/_ab/libqattn_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pb_$v -o run -- \
    python3 $R/$S $A > $R/gpurun_out/pb_$v.log 2>&1
  echo "done $v"
done
