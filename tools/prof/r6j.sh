set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
V=$PWD/tools/prof/_var/libgather.so
R="bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2"
for b in 16384 262144; do
timeout -k 10 240 python -u $R --ring-batch $b > gpurun_out/r6j_inplace_$b.jsonl 2>&1 || exit 1
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $R --ring-batch $b > gpurun_out/r6j_gather_$b.jsonl 2>&1 || exit 1
done
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $R --ring-depth 4 > gpurun_out/r6j_gather_d4.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 240 python -u bench.py --op rx_ring --workload mtu1500 --steps 10 --warmup 2 > gpurun_out/r6j_gather_mtu.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 240 python -u bench.py --op ingress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r6j_gather_ingress_pk.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op ingress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r6j_inplace_ingress_pk.jsonl 2>&1
