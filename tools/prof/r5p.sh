set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_tx_finish.py tests/test_rx_ring.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5p_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r5p_tests.log; exit 1; }
tail -2 gpurun_out/r5p_tests.log
timeout -k 10 180 python -u bench.py --op tx_finish --verify --steps 50 > gpurun_out/r5p_bench_tx_finish.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --op fcs_append --verify --steps 50 > gpurun_out/r5p_bench_fcs_append.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --op tx_checksum --verify --steps 50 > gpurun_out/r5p_bench_tx_checksum.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5p_egress_slots_zipf.jsonl 2>&1
