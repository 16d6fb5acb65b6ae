import sys, time, json
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/compressor-mpc_amd')
import bench
t = time.time()
r = bench.recorded_run_changes(0, int(sys.argv[1]))
print(json.dumps(r), time.time() - t)
