#!/bin/bash
# Build-kernel A/B over the long-horizon configurations (tools/time_build.py,
# 65 536 scenarios, settled): the product library against $OLD.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/bldab.log
for lib in compressor-mpc_amd/cmpc/libcmpc.so $OLD; do
  for c in "par-coop 50 100" "par-cent 100 200" "ser-coop 50 100" "ser-cent 50 100" "ser-ncoop 100" "par-ncoop 100"; do
    set -- $c
    case_=$1; shift
    echo "== $lib $case_" >> gpurun_out/bldab.log
    CMPC_LIBRARY=$PWD/$lib CMPC_TB_VARIANT=rows CMPC_TB_CASE=$case_ timeout -k 10 200 python tools/time_build.py 65536 "$@" >> gpurun_out/bldab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/bldab.log
