#!/bin/bash
# A/B: build kernel priority modes and solve-kernel priority (timing only).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/prio.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so tools/ablate/libcmpc_prio2.so; do
    echo "== $lib" >> gpurun_out/prio.log
    CMPC_TB_VARIANT=rows CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_build.py 65536 50 >> gpurun_out/prio.log 2>&1 || exit $?
  done
  for lib in compressor-mpc_amd/cmpc/libcmpc.so tools/ablate/libcmpc_sprio.so; do
    echo "== $lib" >> gpurun_out/prio.log
    CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_iterate.py 65536 9 >> gpurun_out/prio.log 2>&1 || exit $?
  done
done
cat gpurun_out/prio.log
