#!/bin/bash
# Build a timing variant of libcmpc.so with extra compiler flags into
# ab/<name>/libcmpc.so (git-ignored; it travels to the GPU box with the tree).
# Load it with CMPC_LIBRARY=ab/<name>/libcmpc.so.
#   usage: tools/build_variant.sh NAME "-DFLAG=1 ..."
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EXTRA=$2
W=/tmp/cmpc_variant/$NAME
rm -rf "$W"; mkdir -p "$W/compressor-mpc_amd" "$ROOT/ab/$NAME"
cp -r "$ROOT/include" "$W/include"
cp -r "$ROOT/compressor-mpc_amd/csrc" "$W/compressor-mpc_amd/csrc"
rm -f "$W"/compressor-mpc_amd/csrc/*.o
make -s -j8 -C "$W/compressor-mpc_amd/csrc" OUT="$ROOT/ab/$NAME/libcmpc.so" \
  HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall $EXTRA"
echo "built ab/$NAME/libcmpc.so ($EXTRA)"
