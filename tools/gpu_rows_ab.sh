#!/bin/bash
# Row build kernel: parity tests, then timing of the searched vs packed LDS layout
# and the one-QP-per-wave kernel (one GPU call).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "build" > gpurun_out/ab_t.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/ab_t.log; tail -3 gpurun_out/ab_t.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/ab_time.log
for i in 1 2; do
  echo "== searched" >> gpurun_out/ab_time.log
  timeout -k 10 200 python tools/time_build.py 65536 ${P:-50 100} >> gpurun_out/ab_time.log 2>&1 || exit $?
  echo "== packed" >> gpurun_out/ab_time.log
  CMPC_ROWS_LAYOUT=packed CMPC_TB_VARIANT=rows timeout -k 10 200 python tools/time_build.py 65536 ${P:-50 100} >> gpurun_out/ab_time.log 2>&1 || exit $?
done
cat gpurun_out/ab_time.log
