#!/bin/bash
# small-batch round: parity of the fused/row kernels, then timings and diagnostics
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r4c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/test_$TAG.log
[ $rc -ne 0 ] && exit $rc
OUT=gpurun_out/small_$TAG.txt
timeout -k 10 300 python -u tools/time_small.py c5 c2 b1 c1b1 > $OUT 2>&1 || exit $?
echo "== rows timing p=20 B=4096" >> $OUT
CMPC_LIBRARY=ab/timing/libcmpc.so timeout -k 10 120 python -u tools/rows_timing.py 20 4096 >> $OUT 2>&1 || exit $?
echo "== rows timing p=50 B=1" >> $OUT
CMPC_LIBRARY=ab/timing/libcmpc.so timeout -k 10 120 python -u tools/rows_timing.py 50 1 >> $OUT 2>&1 || exit $?
echo "== build vs p, B=4096" >> $OUT
CMPC_TB_VARIANT=both timeout -k 10 200 python -u tools/time_build.py 4096 2 10 20 50 >> $OUT 2>&1 || exit $?
echo "== build vs p, B=1" >> $OUT
CMPC_TB_VARIANT=both timeout -k 10 200 python -u tools/time_build.py 1 2 10 20 50 >> $OUT 2>&1 || exit $?
echo "== microbench chain" >> $OUT
timeout -k 10 120 tools/microbench_chain >> $OUT 2>&1 || exit $?
echo ALLDONE >> $OUT
# PMC passes on the small-batch kernels (separate runs, kernel trace only)
export TMPDIR=/tmp
pmcs() {  # tag, config, what, counters...
  local t=$1 c=$2 w=$3; shift 3
  timeout -k 10 120 rocprofv3 --kernel-trace -T --kernel-include-regex 'cmpc_' --pmc "$@" \
     -d gpurun_out/pmcsmall_${t} -o run --output-format csv -- python3 tools/pmc_small.py $c $w 20 \
     > gpurun_out/pmcsmall_${t}.log 2>&1
}
for cw in "c5 iterate-rows" "c5 build" "c2 iterate-lane" "c2 step"; do
  set -- $cw
  pmcs "$1_$2_a" $1 $2 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit $?
  pmcs "$1_$2_b" $1 $2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 || exit $?
done
echo PMCDONE >> gpurun_out/small_$TAG.txt
