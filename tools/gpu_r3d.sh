#!/bin/bash
# Round 3: GPU tests, build table, bench line, then the staggered-start A/B
# of the row build kernel (tools/ablate/libcmpc_stag*.so, timing only).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r3d}
bash tools/gpu_r3c.sh $TAG || exit $?
: > gpurun_out/stag_$TAG.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so tools/ablate/libcmpc_stag1.so tools/ablate/libcmpc_stag2.so tools/ablate/libcmpc_stag3.so; do
    echo "== $lib" >> gpurun_out/stag_$TAG.log
    CMPC_TB_VARIANT=rows CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_build.py 65536 50 >> gpurun_out/stag_$TAG.log 2>&1 || exit $?
  done
done
echo ALLDONE
