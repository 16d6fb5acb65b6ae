#!/bin/bash
# Small-batch A/B of library variants (tools/time_small.py); each run has its
# own time limit and a failure ends the script.
#   usage: tools/gpu_small_ab.sh TAG "configs" variant...   (variant "base" = in-tree library)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=$1; CONFS=$2; shift 2
OUT=gpurun_out/small_$TAG.txt
: > $OUT
for v in "$@"; do
  lib=compressor-mpc_amd/cmpc/libcmpc.so
  [ "$v" != base ] && lib=ab/$v/libcmpc.so
  echo "== $v" >> $OUT
  CMPC_LIBRARY=$lib timeout -k 10 240 python -u tools/time_small.py $CONFS >> $OUT 2>&1 || { echo "FAILED rc=$?" >> $OUT; exit 1; }
done
echo ALLDONE >> $OUT
