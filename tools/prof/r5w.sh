set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
V=$PWD/tools/prof/_var/lib1024.so
E="bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2"
timeout -k 10 240 python -u $E > gpurun_out/r5w_e768a.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $E > gpurun_out/r5w_e1024a.jsonl 2>&1 &&
timeout -k 10 240 python -u $E > gpurun_out/r5w_e768b.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $E > gpurun_out/r5w_e1024b.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op egress_packets --bufs slots --workload mtu1500 --steps 10 --warmup 2 > gpurun_out/r5w_e768_mtu.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5w_ring_zipf.jsonl 2>&1
