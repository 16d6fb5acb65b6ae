#!/bin/bash
# One full GPU round: parity tests, smoke, bench, kernel-trace profile, PMC passes.
# Every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r2}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/test_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu --headline-only --markers > gpurun_out/benchprof_$TAG.json 2> gpurun_out/benchprof_$TAG.err || exit $?
# the headline's timed steps and iterate pass cut from that trace (markers)
python3 tools/headline_pass_stats.py gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/benchprof_$TAG.json gpurun_out/bench_$TAG.json gpurun_out/headline_pass_$TAG.csv > gpurun_out/headline_pass_$TAG.txt 2>&1
# the SURVEY configs' own kernels (no headline launches in this trace): their
# --stats averages against the configs section of the bench line above
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cfgprof_$TAG -o run --output-format csv -- python3 bench.py --configs-only --no-cpu > gpurun_out/cfgprof_$TAG.json 2> gpurun_out/cfgprof_$TAG.err || exit $?
pmc() {  # name, counters...   (separate passes, kernel trace only)
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace -T --kernel-include-regex 'cmpc_' \
     --pmc "$@" -d gpurun_out/pmc${TAG}_$name -o run --output-format csv -- \
     python3 bench.py --steps 3 --warmup 1 --no-cpu --headline-only --settle-seconds 0 > gpurun_out/pmc${TAG}_$name.json 2> gpurun_out/pmc${TAG}_$name.err
}
pmc sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit $?
pmc sq2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 || exit $?
pmc fetch FETCH_SIZE || exit $?
pmc write WRITE_SIZE || exit $?
bash tools/gpu_dist_rehearsal.sh > gpurun_out/dist_$TAG.txt 2>&1 || exit $?
echo ALLDONE
