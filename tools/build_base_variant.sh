#!/bin/bash
# Build ab/<name>/libcmpc.so from the tree with one csrc file taken from a git
# revision (the A/B baseline of a kernel change).  ab/ travels to the GPU box
# (it is git-ignored only); delete it once the A/B is recorded.
#   usage: tools/build_base_variant.sh NAME REV FILE(csrc-relative)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2; F=$3
W=/tmp/cmpc_variant/$NAME
rm -rf "$W"; mkdir -p "$W/compressor-mpc_amd" "$ROOT/ab/$NAME"
cp -rp "$ROOT/include" "$W/include"
cp -rp "$ROOT/compressor-mpc_amd/csrc" "$W/compressor-mpc_amd/csrc"
git -C "$ROOT" show "$REV:compressor-mpc_amd/csrc/$F" > "$W/compressor-mpc_amd/csrc/$F"
make -s -j8 -C "$W/compressor-mpc_amd/csrc" OUT="$ROOT/ab/$NAME/libcmpc.so"
echo "built ab/$NAME/libcmpc.so ($F at $REV)"
