#!/bin/bash
# Long-horizon build timing (p = 100, 200; 65 536 scenarios): the product
# library against $OLD, after the build parity tests on the product.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "build or survey" > gpurun_out/lh_t.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/lh_t.log; tail -2 gpurun_out/lh_t.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/lh.log
for lib in compressor-mpc_amd/cmpc/libcmpc.so $OLD; do
  echo "== $lib" >> gpurun_out/lh.log
  for c in par-coop par-cent ser-coop ser-cent; do
    CMPC_TB_VARIANT=both CMPC_TB_CASE=$c CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_build.py 65536 100 >> gpurun_out/lh.log 2>&1 || exit $?
  done
  CMPC_TB_VARIANT=wave CMPC_TB_CASE=par-cent CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_build.py 65536 200 >> gpurun_out/lh.log 2>&1 || exit $?
done
CMPC_TB_VARIANT=rows CMPC_TB_CASE=par-cent timeout -k 10 200 python tools/time_build.py 65536 200 >> gpurun_out/lh.log 2>&1
CMPC_TB_VARIANT=rows CMPC_TB_CASE=par-cent timeout -k 10 200 python tools/time_build.py 1024 200 >> gpurun_out/lh.log 2>&1
CMPC_TB_VARIANT=wave CMPC_TB_CASE=par-cent timeout -k 10 200 python tools/time_build.py 1024 200 >> gpurun_out/lh.log 2>&1
grep -v amdgpu.ids gpurun_out/lh.log
