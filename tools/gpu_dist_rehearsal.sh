#!/bin/bash
# Rehearse bench.py's multi-process launch on a one-GPU box: two ranks under
# torch.distributed.run share the GPU, the barrier / max-over-ranks run on
# gloo (RCCL refuses two ranks on one device).  The 8-GPU RCCL run is the
# driver's.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
  --batch 16384 --no-cpu --dist-backend gloo > gpurun_out/dist2.json 2> gpurun_out/dist2.err
rc=$?; echo "dist rc=$rc"; tail -c 600 gpurun_out/dist2.json; exit $rc
