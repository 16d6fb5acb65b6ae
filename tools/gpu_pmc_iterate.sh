#!/bin/bash
# PMC of the iterate kernel in the bench's step loop (tools/pmc_iterate.py),
# with and without the applied move, for the in-tree library and (if built)
# ab/r4/libcmpc.so.  Separate --pmc passes, kernel trace only.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag lib mode counters...
  local t=$1 lib=$2 mode=$3; shift 3
  CMPC_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex 'cmpc_solve' --pmc "$@" \
     -d gpurun_out/pmcit_$t -o run --output-format csv -- python3 tools/pmc_iterate.py $mode 24 \
     > gpurun_out/pmcit_$t.log 2>&1
}
for lib in cur r4; do
  L=compressor-mpc_amd/cmpc/libcmpc.so; [ $lib = r4 ] && L=ab/r4/libcmpc.so
  for mode in move nomove; do
    run ${lib}_${mode}_a $L $mode SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM || exit $?
    run ${lib}_${mode}_b $L $mode SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F64 || exit $?
  done
done
echo PMCDONE
