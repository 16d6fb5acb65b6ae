#!/bin/bash
# Rehearse bench.py's multi-process launch on a one-GPU box with the driver's
# plain command line (no torchrun on it): `bench.py --gpus 2` starts the two
# ranks itself (a torch.distributed.run child); they share the GPU, the
# barrier / max-over-ranks run on gloo (RCCL refuses two ranks on one device).
# Then `--gpus 8` under RCCL must refuse to run on one visible GPU.  The 8-GPU
# RCCL run is the driver's.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --batch 16384 --no-cpu \
  --dist-backend gloo > gpurun_out/dist2.json 2> gpurun_out/dist2.err
rc=$?; echo "dist rc=$rc"; tail -c 400 gpurun_out/dist2.json; echo
[ $rc -eq 0 ] || exit $rc
python3 -c "import json,sys; d=json.loads(open('gpurun_out/dist2.json').read().splitlines()[-1]); \
print('n_gpus', d['n_gpus'], 'launch', d['launch'], 'rank_ms_per_step', d['rank_ms_per_step']); \
sys.exit(0 if d['n_gpus'] == 2 and len(d['rank_ms_per_step']) == 2 else 1)" || exit 1
timeout -k 10 120 python3 bench.py --gpus 8 --steps 2 --no-cpu > gpurun_out/dist8.json 2> gpurun_out/dist8.err
rc8=$?; echo "gpus 8 on this box: rc=$rc8 ($(tail -1 gpurun_out/dist8.err))"
[ $rc8 -ne 0 ] && [ $rc8 -ne 124 ] && [ $rc8 -ne 137 ] || exit 1
exit 0
