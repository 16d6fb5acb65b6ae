#!/bin/bash
# PMC of the row build kernel for two configurations (time_build.py, p = 50):
# instruction mix, LDS and occupancy counters per case, one pass each.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in ${CASES:-par-coop ser-coop}; do
  CMPC_TB_VARIANT=rows CMPC_TB_CASE=$c CMPC_TB_SETTLE=0.05 timeout -s KILL 120 rocprofv3 --kernel-trace \
    --kernel-include-regex 'cmpc_build_rows' \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU \
    -d gpurun_out/pmcc_$c -o run --output-format csv -- python3 tools/time_build.py 65536 ${P:-50} > gpurun_out/pmcc_$c.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections, os
for c in os.environ.get("CASES", "par-coop ser-coop").split():
    f = f"gpurun_out/pmcc_{c}/run_counter_collection.csv"
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(c, {k: round(sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
