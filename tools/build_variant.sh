#!/bin/bash
# Build a timing variant of libcmpc.so with extra compiler flags into
# ab/<name>/libcmpc.so (git-ignored; it travels to the GPU box with the tree).
# Load it with CMPC_LIBRARY=ab/<name>/libcmpc.so.
#   usage: tools/build_variant.sh NAME "-DFLAG=1 ..." [HEADER ...]
# With HEADERs (csrc-relative), the in-tree objects are reused and only the
# objects that depend on those headers are rebuilt with the extra flags.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; EXTRA=$2; shift 2 || true
W=/tmp/cmpc_variant/$NAME
rm -rf "$W"; mkdir -p "$W/compressor-mpc_amd" "$ROOT/ab/$NAME"
cp -rp "$ROOT/include" "$W/include"
cp -rp "$ROOT/compressor-mpc_amd/csrc" "$W/compressor-mpc_amd/csrc"
if [ $# -eq 0 ]; then
  rm -f "$W"/compressor-mpc_amd/csrc/*.o
else
  for h in "$@"; do touch "$W/compressor-mpc_amd/csrc/$h"; done
fi
make -s -j8 -C "$W/compressor-mpc_amd/csrc" OUT="$ROOT/ab/$NAME/libcmpc.so" \
  HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall $EXTRA"
echo "built ab/$NAME/libcmpc.so ($EXTRA)"
