#!/bin/bash
# PMC passes (kernel-trace only, never with sys/runtime tracing) on the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-pmc}
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace -T --kernel-include-regex 'cmpc_(build|solve)_kernel' \
     --pmc "$@" -d gpurun_out/${TAG}_$name -o run --output-format csv -- \
     python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err
  echo "$name rc=$?"
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64
run fetch FETCH_SIZE
run write WRITE_SIZE
echo PMCDONE
