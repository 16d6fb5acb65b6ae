cd "${GRAFT_REPO_ROOT:-/root/repo}"
for c in par-coop ser-coop ser-cent; do
  for lib in compressor-mpc_amd/cmpc/libcmpc.so tools/ablate/libcmpc_wpe2.so; do
    echo "$c $lib $(CMPC_TB_VARIANT=rows CMPC_TB_CASE=$c CMPC_LIBRARY=$PWD/$lib timeout -k 10 120 python tools/time_build.py 65536 50 100 2>/dev/null | tr '\n' ' ')"
  done
done
