set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6w
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6w/smoke.log 2>&1 && tail -1 gpurun_out/r6w/smoke.log &&
timeout -k 10 300 python -u bench.py > gpurun_out/r6w/bench_default.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --workload zipf64_1500 --verify --steps 20 > gpurun_out/r6w/bench_zipf.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --workload jumbo9000 --verify --steps 20 > gpurun_out/r6w/bench_jumbo.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_verify --verify --steps 50 > gpurun_out/r6w/bench_rx_verify.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op tx_finish --verify --steps 50 > gpurun_out/r6w/bench_tx_finish.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op fcs_append --verify --steps 50 > gpurun_out/r6w/bench_fcs_append.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op tx_checksum --verify --steps 50 > gpurun_out/r6w/bench_tx_checksum.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r6w/bench_ring_zipf.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r6w/bench_egress_zipf.jsonl 2>&1
