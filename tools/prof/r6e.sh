set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_tx_finish.py tests/test_rx_ring.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6e_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6e_tests.log; exit 1; }
tail -1 gpurun_out/r6e_tests.log
timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r6e_parts.json 2>&1 &&
timeout -k 10 180 python -u bench.py --op tx_finish --verify --steps 50 --no-cpu-baseline > gpurun_out/r6e_txf.jsonl 2>&1
