cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
: > gpurun_out/wpg.log
for c in ser-coop ser-cent par-coop par-cent; do
  for w in 4 2; do
    echo "WPG=$w" >> gpurun_out/wpg.log
    CMPC_ROWS_WPG=$w CMPC_TB_VARIANT=rows CMPC_TB_CASE=$c timeout -k 10 200 python tools/time_build.py 65536 100 >> gpurun_out/wpg.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/wpg.log
