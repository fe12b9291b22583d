#!/bin/bash
# round 6: int8 forward, partial scalar dequantisation / S conversion (A/B, alternating)
set -o pipefail
export QATTN_AB_MODES=qf
{
for v in default nslp dq1 dq2 s4 s8 dq1s4 dq1s4 s8 s4 dq2 dq1 nslp default default dq1 dq2 nslp; do
  bash tools/ab_run.sh tools/ab_time.py $v 2>&1 | grep -v amdgpu.ids | grep "pv=" | sed "s/^/$v /" || exit 1
done
} > gpurun_out/r06a_ab.log 2>&1 || { echo AB FAILED; tail -20 gpurun_out/r06a_ab.log; exit 1; }
cat gpurun_out/r06a_ab.log
