#!/bin/bash
# PMC passes on the build kernel alone (kernel trace only; one counter group per pass).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-pb}
P=${2:-50}
export TMPDIR=/tmp
pmc() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace -T --kernel-include-regex 'cmpc_build' \
     --pmc "$@" -d gpurun_out/pmc${TAG}_$name -o run --output-format csv -- \
     python3 tools/run_build.py $P > gpurun_out/pmc${TAG}_$name.log 2>&1
}
pmc a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit $?
pmc b SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE || exit $?
pmc d FETCH_SIZE || exit $?
pmc e WRITE_SIZE || exit $?
pmc c SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP SQ_INSTS_VALU_FMA_F64 SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_MEM_VIOLATIONS SQ_WAIT_INST_ANY || exit $?
echo PMCDONE
