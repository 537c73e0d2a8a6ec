set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5i
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5i/egress -o egress --output-format csv -- python3 bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 5 --warmup 1 > gpurun_out/r5i/egress.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5i/ingress -o ingress --output-format csv -- python3 bench.py --op ingress_packets --bufs slots --workload zipf64_1500 --steps 5 --warmup 1 > gpurun_out/r5i/ingress.log 2>&1
