set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5o
timeout -k 10 300 python -u bench.py > gpurun_out/r5o/bench_default.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --workload zipf64_1500 --verify --steps 20 > gpurun_out/r5o/bench_zipf.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --op rx_verify --verify --steps 50 > gpurun_out/r5o/bench_rx_verify.jsonl 2>&1 &&
timeout -k 10 240 python -u bench.py --workload jumbo9000 --verify --steps 20 > gpurun_out/r5o/bench_jumbo.jsonl 2>&1
