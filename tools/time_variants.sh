#!/bin/bash
# Time the build kernel at p=50 for the product library and each ablation variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for lib in compressor-mpc_amd/cmpc/libcmpc.so tools/ablate/libcmpc_exp5.so tools/ablate/libcmpc_exp6.so; do
  echo "== $lib" >> gpurun_out/variants.log
  CMPC_LIBRARY=$PWD/$lib timeout -k 10 120 python tools/time_build.py 65536 50 >> gpurun_out/variants.log 2>&1 || exit $?
done
