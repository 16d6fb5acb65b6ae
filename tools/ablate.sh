#!/bin/bash
# Build timing-only ablation variants of libcmpc.so (CMPC_EXP=1..4, results
# are NOT valid) into /tmp and time the build kernel with each.
set -e
cd "$(dirname "$0")/../compressor-mpc_amd/csrc"
for e in ${EXPS:-1 2 3 4 5 6}; do
  mkdir -p ../../tools/ablate
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -DCMPC_EXP=$e -c cmpc_kernels.hip -o /tmp/k$e.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/ablate/libcmpc_exp$e.so /tmp/k$e.o cmpc_abi.o plant.o
done
