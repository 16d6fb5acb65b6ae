#!/bin/bash
# Build-kernel variants: parity tests then timing (one GPU call).
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "build" > gpurun_out/rows_t1.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/rows_t1.log; tail -5 gpurun_out/rows_t1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/time_build.py 65536 50 100 > gpurun_out/rows_time.log 2>&1
rc=$?; cat gpurun_out/rows_time.log; exit $rc
