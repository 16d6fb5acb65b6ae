#!/bin/bash
# Time the row-layout build kernel at p=50 for the product library and each ablation variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out; : > gpurun_out/rxvariants.log
for lib in compressor-mpc_amd/cmpc/libcmpc.so tools/ablate/libcmpc_rx*.so; do
  echo "== $lib" >> gpurun_out/rxvariants.log
  CMPC_TB_VARIANT=rows CMPC_LIBRARY=$PWD/$lib timeout -k 10 120 python tools/time_build.py 65536 ${P:-2 50} >> gpurun_out/rxvariants.log 2>&1 || exit $?
done
cat gpurun_out/rxvariants.log
