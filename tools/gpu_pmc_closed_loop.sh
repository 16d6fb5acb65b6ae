#!/bin/bash
# PMC passes over the closed loop's producer and observer kernels
# (tools/run_closed_loop.py, 65 536 scenarios): kernel trace + stats, then
# one counter set per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-clpmc}
RUN="python3 tools/run_closed_loop.py par coop --batch 65536 --steps 20 --perturb 0.002"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv -- $RUN > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
pmc() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex 'cmpc_produce|cmpc_obs' \
    --pmc "$@" -d gpurun_out/${TAG}_$name -o run --output-format csv -- $RUN > gpurun_out/${TAG}_$name.log 2>&1
}
pmc sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit $?
pmc sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE || exit $?
pmc fetch FETCH_SIZE || exit $?
pmc write WRITE_SIZE || exit $?
echo ALLDONE
