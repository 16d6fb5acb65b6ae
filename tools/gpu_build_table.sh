#!/bin/bash
# Re-measure DESIGN §3.0's build table: both build kernels, six configurations,
# p = 20, 50, 100 (and par-cent p = 200), 65 536 scenarios, settled clock.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/btab.log
for c in par-coop par-ncoop par-cent ser-coop ser-ncoop ser-cent; do
  echo "== $c" >> gpurun_out/btab.log
  CMPC_TB_VARIANT=both CMPC_TB_CASE=$c timeout -k 10 240 python tools/time_build.py 65536 20 50 100 >> gpurun_out/btab.log 2>&1 || exit $?
done
echo "== par-cent p200" >> gpurun_out/btab.log
CMPC_TB_VARIANT=both CMPC_TB_CASE=par-cent timeout -k 10 240 python tools/time_build.py 65536 200 >> gpurun_out/btab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/btab.log
