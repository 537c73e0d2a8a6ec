set -o pipefail
cd $GRAFT_REPO_ROOT
for B in 262144 1048576; do
  for OP in egress_packets ingress_packets; do
    timeout -k 10 240 python -u bench.py --op $OP --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 --ring-batch $B --ring-depth 2 > gpurun_out/r5j_${OP}_${B}.jsonl 2>&1 || exit 1
  done
  timeout -k 10 240 python -u bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2 --ring-batch $B --ring-depth 2 > gpurun_out/r5j_rx_ring_${B}.jsonl 2>&1 || exit 1
done
echo done
