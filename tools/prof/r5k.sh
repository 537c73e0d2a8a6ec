set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5k
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k/ring -o ring --output-format csv -- python3 bench.py --op rx_ring --workload zipf64_1500 --steps 5 --warmup 1 --ring-batch 1048576 --ring-depth 1 > gpurun_out/r5k/ring.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5k/ringmtu -o ringmtu --output-format csv -- python3 bench.py --op rx_ring --workload mtu1500 --steps 5 --warmup 1 --ring-batch 1048576 --ring-depth 1 > gpurun_out/r5k/ringmtu.log 2>&1
