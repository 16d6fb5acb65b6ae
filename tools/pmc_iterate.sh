#!/bin/bash
# PMC pass on the iterate kernel (repeated batch, K = 1 and K = 9): VALU/SALU
# instructions per wave and SIMD busy, for the per-iteration cost.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 1 9; do
  CMPC_TB_SETTLE=0 timeout -k 10 300 rocprofv3 --kernel-trace -T --kernel-include-regex 'cmpc_solve' \
     --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_ACTIVE_INST_ANY \
     -d gpurun_out/pmcit_$K -o run --output-format csv -- python3 tools/time_iterate.py 65536 $K > gpurun_out/pmcit_$K.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
for K in (1, 9):
    f = glob.glob(f"gpurun_out/pmcit_{K}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    d = {k: sum(v) / len(v) for k, v in acc.items()}
    w = d.get("SQ_WAVES", 1)
    print(f"K={K}: launches {len(acc['SQ_WAVES'])}  " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(d.items())) +
          f"  VALU/wave {d['SQ_INSTS_VALU']/w:.0f} SALU/wave {d['SQ_INSTS_SALU']/w:.0f} F64FMA/wave {d['SQ_INSTS_VALU_FMA_F64']/w:.0f}")
PY
