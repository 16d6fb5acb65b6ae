#!/bin/bash
# Timing-only ablation variants of the row-layout build kernel (CMPC_RX=1..4;
# results are NOT valid) -> tools/ablate/libcmpc_rx<e>.so
set -e
cd "$(dirname "$0")/../compressor-mpc_amd/csrc"
mkdir -p ../../tools/ablate
OBJS="cmpc_kernels.o rows_layout.o cmpc_abi.o plant.o produce.o coupled.o observer.o sim.o"
for e in ${EXPS:-1 2 3 4}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -DCMPC_RX=$e -c build_rows.hip -o /tmp/rx$e.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/ablate/libcmpc_rx$e.so /tmp/rx$e.o $OBJS
done
