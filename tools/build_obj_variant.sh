#!/bin/bash
# ab/<name>/libcmpc.so with ONE object rebuilt with extra compiler flags (the
# rest from the tree): an A/B of, e.g., a scheduler option on the solver's
# object only.  ab/ travels to the GPU box; delete it once the A/B is recorded.
#   usage: tools/build_obj_variant.sh NAME OBJECT.o "EXTRA FLAGS"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; OBJ=$2; EXTRA=$3
W=/tmp/cmpc_variant/$NAME
rm -rf "$W"; mkdir -p "$W/compressor-mpc_amd" "$ROOT/ab/$NAME"
cp -rp "$ROOT/include" "$W/include"
cp -rp "$ROOT/compressor-mpc_amd/csrc" "$W/compressor-mpc_amd/csrc"
rm -f "$W/compressor-mpc_amd/csrc/$OBJ"
make -s -j8 -C "$W/compressor-mpc_amd/csrc" OUT="$ROOT/ab/$NAME/libcmpc.so" \
  SOLVERFLAGS="-mllvm -simplifycfg-sink-common=false $EXTRA"
echo "built ab/$NAME/libcmpc.so ($OBJ with $EXTRA)"
