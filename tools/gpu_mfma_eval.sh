#!/bin/bash
# Round 3: GPU tests, the FP64-MFMA microbenchmark (tools/microbench_hybrid,
# V4 = A^4-blocked P chain + Markov + Gram on MFMA) and the MFMA/VALU PMC
# counters of the product build at cent-par p = 200 (B = 1024, 65536) and of
# the microbenchmark's variants.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r3b}
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/test_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 tools/microbench_hybrid > gpurun_out/mb_$TAG.txt 2>&1 || exit $?
CNT="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for B in 1024 65536; do
  CMPC_TB_CASE=par-cent timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex 'cmpc_build' --pmc $CNT \
    -d gpurun_out/pmc${TAG}_cent200_$B -o run --output-format csv -- python3 tools/time_build.py $B 200 \
    > gpurun_out/pmc${TAG}_cent200_$B.txt 2>&1 || exit $?
done
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $CNT -d gpurun_out/pmc${TAG}_mb -o run --output-format csv -- \
  tools/microbench_hybrid > gpurun_out/pmc${TAG}_mb.txt 2>&1 || exit $?
echo ALLDONE
