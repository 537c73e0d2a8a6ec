set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
for G in 56 60; do
LNETO_AMD_LIB=$PWD/tools/prof/_var/libg$G.so timeout -k 10 600 python -u -m pytest tests/test_rx_verify.py tests/test_tx_finish.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r6r_tests_g$G.log 2>&1 || { echo TESTS_FAILED $G; tail -30 gpurun_out/r6r_tests_g$G.log; exit 1; }
tail -1 gpurun_out/r6r_tests_g$G.log
done
B="bench.py --op rx_verify --steps 50 --no-cpu-baseline"
T="bench.py --op tx_finish --steps 50 --no-cpu-baseline"
for i in 1 2; do
for G in 48 56 60; do
if [ $G = 48 ]; then E=""; else E="LNETO_AMD_LIB=$PWD/tools/prof/_var/libg$G.so"; fi
env $E timeout -k 10 180 python -u $B > gpurun_out/r6r_rxv_g${G}_$i.jsonl 2>&1 || exit 1
env $E timeout -k 10 180 python -u $T > gpurun_out/r6r_txf_g${G}_$i.jsonl 2>&1 || exit 1
done
done
