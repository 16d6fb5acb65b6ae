#!/bin/bash
# Build a variant of libcmpc.so with extra preprocessor defines on the row
# build kernel and its layout (e.g. -DCMPC_ROWS_WPS=4) into
# tools/ablate/libcmpc_NAME.so, for A/B timing with CMPC_LIBRARY=...
#   usage: tools/build_variant.sh NAME "-DFOO=1 -DBAR=2" [sources...]
# (default sources: build_rows.hip rows_layout.cpp; e.g. cmpc_kernels.hip for the solver)
set -e
name=$1; defs=$2
cd "$(dirname "$0")/../compressor-mpc_amd/csrc"
make -s -j8
mkdir -p ../../tools/ablate
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off $defs"
shift 2
srcs=${*:-build_rows.hip rows_layout.cpp}
vobjs=""; skip=""
for src in $srcs; do
  o=/tmp/v_${name}_${src%.*}.o
  extra=""
  case $src in cmpc_kernels.hip|coupled.hip) extra="-mllvm -simplifycfg-sink-common=false";; esac
  /opt/rocm/bin/hipcc $F $extra -c $src -o $o
  vobjs="$vobjs $o"; skip="$skip -e ^${src%.*}.o$"
done
objs=$(ls *.o | grep -v $skip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../tools/ablate/libcmpc_$name.so $vobjs $objs
echo "built tools/ablate/libcmpc_$name.so"
