set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_rx_verify.py tests/test_tx_finish.py tests/test_rx_ring.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6b_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6b_tests.log; exit 1; }
tail -1 gpurun_out/r6b_tests.log
timeout -k 10 180 python -u bench.py --op rx_verify --verify --steps 50 --no-cpu-baseline > gpurun_out/r6b_rxv.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --op tx_finish --verify --steps 50 --no-cpu-baseline > gpurun_out/r6b_txf.jsonl 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-trace -d gpurun_out/r6b_pmc -o pmc --output-format csv -- python3 bench.py --op rx_verify --no-cpu-baseline --no-slice16m --prewarm-s 0 --steps 5 --warmup 1 > gpurun_out/r6b_pmc.log 2>&1
