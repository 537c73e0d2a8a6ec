set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
LNETO_AMD_LIB=$PWD/tools/prof/_var/lib_56_64.so timeout -k 10 600 python -u -m pytest tests/test_tx_finish.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6u_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6u_tests.log; exit 1; }
tail -1 gpurun_out/r6u_tests.log
B="bench.py --op rx_verify --steps 50 --no-cpu-baseline"
T="bench.py --op tx_finish --steps 50 --no-cpu-baseline"
for i in 1 2; do
timeout -k 10 180 python -u $B > gpurun_out/r6u_rxv_56_$i.jsonl 2>&1 || exit 1
LNETO_AMD_LIB=$PWD/tools/prof/_var/lib_52_60.so timeout -k 10 180 python -u $B > gpurun_out/r6u_rxv_52_$i.jsonl 2>&1 || exit 1
timeout -k 10 180 python -u $T > gpurun_out/r6u_txf_60_$i.jsonl 2>&1 || exit 1
LNETO_AMD_LIB=$PWD/tools/prof/_var/lib_56_64.so timeout -k 10 180 python -u $T > gpurun_out/r6u_txf_64_$i.jsonl 2>&1 || exit 1
done
