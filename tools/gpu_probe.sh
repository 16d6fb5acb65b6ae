#!/bin/bash
# Build-kernel instruction-cost probe (tools/ablate/libcmpc_px{4,5,6}.so: 200
# extra int / 64-bit move / FP64 FMA VALU instructions per group, results
# unchanged) against the product, twice; then the two-rank rehearsal of
# bench.py's multi-process path (gloo, both ranks on the one GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/probe.log
for i in 1 2; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so tools/ablate/libcmpc_px4.so tools/ablate/libcmpc_px5.so tools/ablate/libcmpc_px6.so; do
    echo "== $lib" >> gpurun_out/probe.log
    CMPC_TB_VARIANT=rows CMPC_LIBRARY=$PWD/$lib timeout -k 10 200 python tools/time_build.py 65536 50 >> gpurun_out/probe.log 2>&1 || exit $?
  done
done
bash tools/gpu_dist_rehearsal.sh || exit $?
echo ALLDONE
