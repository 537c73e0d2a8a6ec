set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_tx_finish.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6p_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6p_tests.log; exit 1; }
tail -12 gpurun_out/r6p_tests.log
