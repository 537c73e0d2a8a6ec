set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5x_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5x_tests.log; exit 1; }
tail -1 gpurun_out/r5x_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5x_smoke.log 2>&1 && tail -2 gpurun_out/r5x_smoke.log &&
timeout -k 10 240 python -u bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2 > gpurun_out/r5x_egress_zipf.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --op tx_finish --verify --steps 50 --no-cpu-baseline > gpurun_out/r5x_txf.jsonl 2>&1
