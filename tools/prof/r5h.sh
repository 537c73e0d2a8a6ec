set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_rx_ring.py tests/test_rx_verify.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5h_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5h_tests.log; exit 1; }
tail -2 gpurun_out/r5h_tests.log
timeout -k 10 240 python -u bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5h_egress_slots_zipf.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op egress_packets --bufs slots --workload mtu1500 --steps 10 --warmup 2 > gpurun_out/r5h_egress_slots_mtu.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op ingress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5h_ingress_slots_zipf.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --steps 50 --warmup 5 --op rx_verify --no-cpu-baseline --verify > gpurun_out/r5h_bench_rx_verify.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5h_ring_zipf_zc.jsonl 2>&1
