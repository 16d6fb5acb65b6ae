#!/bin/bash
# A/B of the coupled iterate's G_ext layout (config 4's 64-sub-controller
# system at world 1): the in-tree library with the QP-blocked layout against
# ab/elem/libcmpc.so (the element-major kernel) fed element-major data,
# alternating.   usage: tools/gpu_coupled_layout_ab.sh [ROUNDS]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/layout_ab.txt; : > $OUT
for i in $(seq ${1:-3}); do
  for v in blocked elem; do
    if [ $v = blocked ]; then L=""; else L=ab/elem/libcmpc.so; fi
    CMPC_LIBRARY=$L timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, 'compressor-mpc_amd')
import cmpc.coupled as cc
if sys.argv[1] == 'elem':
    cc.g_ext_blocked = lambda em: em.reshape(-1)  # the previous layout, [E][nqp]
r = cc.run_coupled_bench(0, 1, 0, S_local=64, S_total=64, B=4096, steps=10, settle_seconds=0.25)
print(sys.argv[1], sys.argv[2], 'ms_per_step %.4f iterate_ms %.4f G_ext_hbm_frac %.3f ok %.3f' % (r['elapsed_s'] / r['steps'] * 1e3, r['iterate_kernel_ms'], r['G_ext_hbm_frac'], r['qp_status_ok_fraction']))
" $v $i >> $OUT 2> gpurun_out/layout_$v$i.err || exit $?
  done
done
cat $OUT
