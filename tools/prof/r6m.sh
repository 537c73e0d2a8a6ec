set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
V=$PWD/tools/prof/_var/libpf8.so
timeout -k 10 600 python -u -m pytest tests/test_rx_verify.py tests/test_rx_ring.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6m_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6m_tests.log; exit 1; }
tail -1 gpurun_out/r6m_tests.log
B="bench.py --op rx_verify --steps 50 --no-cpu-baseline"
timeout -k 10 180 python -u $B > gpurun_out/r6m_rxv12_1.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 180 python -u $B > gpurun_out/r6m_rxv8_1.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 180 python -u $B > gpurun_out/r6m_rxv8_2.jsonl 2>&1 &&
timeout -k 10 180 python -u $B > gpurun_out/r6m_rxv12_2.jsonl 2>&1 &&
timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r6m_parts12.json 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r6m_parts8.json 2>&1 &&
R="bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2" &&
timeout -k 10 240 python -u $R > gpurun_out/r6m_ring12.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $R > gpurun_out/r6m_ring8.jsonl 2>&1
