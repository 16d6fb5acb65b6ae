#!/bin/bash
# Build a variant of libcmpc.so with extra preprocessor defines on the row
# build kernel and its layout (e.g. -DCMPC_ROWS_WPS=4) into
# tools/ablate/libcmpc_NAME.so, for A/B timing with CMPC_LIBRARY=...
#   usage: tools/build_variant.sh NAME "-DFOO=1 -DBAR=2"
set -e
name=$1; defs=$2
cd "$(dirname "$0")/../compressor-mpc_amd/csrc"
make -s -j8
mkdir -p ../../tools/ablate
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off $defs"
/opt/rocm/bin/hipcc $F -c build_rows.hip -o /tmp/v_${name}_br.o
/opt/rocm/bin/hipcc $F -c rows_layout.cpp -o /tmp/v_${name}_rl.o
objs=$(ls *.o | grep -v -e '^build_rows.o$' -e '^rows_layout.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/ablate/libcmpc_$name.so /tmp/v_${name}_br.o /tmp/v_${name}_rl.o $objs
echo "built tools/ablate/libcmpc_$name.so"
