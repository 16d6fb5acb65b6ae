#!/bin/bash
# Build-kernel time for every plant/controller type at p = 20, 50, 100 (AUTO and both kernels).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/cfgsweep.log
for c in par-coop par-ncoop par-cent ser-coop ser-ncoop ser-cent; do
  CMPC_TB_CASE=$c timeout -k 10 200 python tools/time_build.py 65536 20 50 100 >> gpurun_out/cfgsweep.log 2>&1 || exit $?
done
cat gpurun_out/cfgsweep.log
