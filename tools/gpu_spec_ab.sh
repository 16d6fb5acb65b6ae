cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
true
ROUNDS=3 CONFIGS=1 bash tools/gpu_ab_multi.sh spec orig
