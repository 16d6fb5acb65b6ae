#!/bin/bash
# Iterate-kernel A/B: the full GPU suite on the product library, then
# cmpc_iterate timing (K = 9 and 1, settled) of the product and of $LIBS.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_t.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/iter_t.log; tail -3 gpurun_out/iter_t.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/iter_time.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    for K in 9 1; do
      echo "== $lib" >> gpurun_out/iter_time.log
      CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_iterate.py 65536 $K >> gpurun_out/iter_time.log 2>&1 || exit $?
    done
  done
done
grep -v amdgpu.ids gpurun_out/iter_time.log
