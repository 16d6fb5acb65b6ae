#!/bin/bash
# Row build kernel: horizon sweep (fixed vs per-step cost) and ablation libs at p = 50.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/psweep.log
CMPC_TB_VARIANT=rows timeout -k 10 200 python tools/time_build.py 65536 2 10 25 50 >> gpurun_out/psweep.log 2>&1 || exit $?
for lib in $LIBS; do
  echo "== $lib" >> gpurun_out/psweep.log
  CMPC_TB_VARIANT=rows CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_build.py 65536 2 50 >> gpurun_out/psweep.log 2>&1 || exit $?
done
cat gpurun_out/psweep.log
