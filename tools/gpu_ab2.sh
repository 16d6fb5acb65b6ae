#!/bin/bash
# Build-kernel A/B with parity: the build parity tests on the product library
# and on every library in $LIBS, then build timing of all of them, twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/ab_t.log
[ "${TESTK:-build}" = none ] || for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
  echo "== $lib" >> gpurun_out/ab_t.log
  CMPC_LIBRARY=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-build}" >> gpurun_out/ab_t.log 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/ab_t.log
  [ $rc -eq 0 ] || exit $rc
done
: > gpurun_out/ab_time.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    echo "== $lib" >> gpurun_out/ab_time.log
    CMPC_TB_VARIANT=rows CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_build.py 65536 ${P:-50} >> gpurun_out/ab_time.log 2>&1 || exit $?
  done
done
cat gpurun_out/ab_time.log
