set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-slice16m > gpurun_out/r5b_bench_mtu1500.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --steps 50 --warmup 5 --op rx_verify --no-cpu-baseline --verify > gpurun_out/r5b_bench_rx_verify.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --workload zipf64_1500 --no-cpu-baseline > gpurun_out/r5b_bench_zipf.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --workload zipf64_1500 --short-frames --no-cpu-baseline > gpurun_out/r5b_bench_zipf_short.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --steps 50 --warmup 3 --workload jumbo9000 --no-cpu-baseline > gpurun_out/r5b_bench_jumbo.jsonl 2>&1 &&
timeout -k 10 300 ./tools/ubench/call_latency > gpurun_out/r5b_call_latency.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5b_ring_zipf_zc.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2 --ring-copy > gpurun_out/r5b_ring_zipf_copy.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_ring --workload mtu1500 --steps 10 --warmup 2 > gpurun_out/r5b_ring_mtu_zc.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op ingress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5b_ingress_slots_zipf.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5b_egress_slots_zipf.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op egress_packets --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5b_egress_own_zipf.jsonl 2>&1
