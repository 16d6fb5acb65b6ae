#!/bin/bash
# Solve-kernel A/B: the GPU parity suite (product library), then iterate
# timing (coop p=50, K=9) and the SURVEY config table for the product library
# and each library in $LIBS, in one GPU call.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sab_t.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/sab_t.log; tail -3 gpurun_out/sab_t.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/sab_time.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    echo "== $lib" >> gpurun_out/sab_time.log
    CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_iterate.py 65536 9 >> gpurun_out/sab_time.log 2>&1 || exit $?
  done
done
for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
  echo "== $lib" >> gpurun_out/sab_time.log
  CMPC_LIBRARY=$PWD/$lib timeout -k 10 300 python tools/time_survey_configs.py >> gpurun_out/sab_time.log 2>&1 || exit $?
done
cat gpurun_out/sab_time.log
