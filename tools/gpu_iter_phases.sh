#!/bin/bash
# Iterate-kernel phase timing (tools/time_iterate_phases.py) for the product
# library and each library in $LIBS; the GPU suite on each of $TESTLIBS first.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/iph.log
for lib in ${TESTLIBS:-}; do
  CMPC_LIBRARY=$PWD/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iph_t.log 2>&1
  rc=$?; echo "$lib pytest rc=$rc: $(tail -1 gpurun_out/iph_t.log)" | tee -a gpurun_out/iph.log
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so $LIBS; do
    echo "== $lib" >> gpurun_out/iph.log
    CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_iterate_phases.py >> gpurun_out/iph.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/iph.log
