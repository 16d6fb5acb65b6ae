mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/test_r4f.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/time_small.py c5 c2 b1 c1b1 > gpurun_out/small_r4f.txt 2>&1 || exit $?
echo "== hand depth 1" >> gpurun_out/small_r4f.txt
CMPC_LIBRARY=ab/hand1/libcmpc.so timeout -k 10 300 python -u tools/time_small.py c5 b1 c1b1 >> gpurun_out/small_r4f.txt 2>&1 || exit $?
bash tools/gpu_b1_trace.sh r4f
