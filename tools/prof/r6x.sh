set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_rx_verify.py tests/test_tx_finish.py -x -q --timeout 300 --timeout-method thread -m gpu -k "batch_sizes" > gpurun_out/r6x_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6x_tests.log; exit 1; }
tail -2 gpurun_out/r6x_tests.log
