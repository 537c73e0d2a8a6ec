set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
V=$PWD/tools/prof/_var/lib4k.so
R="bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2"
E="bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2"
timeout -k 10 300 python -u -m pytest tests/test_rx_ring.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r6a_tests.log 2>&1 || { tail -20 gpurun_out/r6a_tests.log; exit 1; }
tail -1 gpurun_out/r6a_tests.log
for i in 1 2; do
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $R > gpurun_out/r6a_ring4k_$i.jsonl 2>&1 || exit 1
timeout -k 10 240 python -u $R > gpurun_out/r6a_ring2m_$i.jsonl 2>&1 || exit 1
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $E > gpurun_out/r6a_eg4k_$i.jsonl 2>&1 || exit 1
timeout -k 10 240 python -u $E > gpurun_out/r6a_eg2m_$i.jsonl 2>&1 || exit 1
done
for i in 3; do
timeout -k 10 240 python -u $R > gpurun_out/r6a_ring2m_$i.jsonl 2>&1 || exit 1
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $R > gpurun_out/r6a_ring4k_$i.jsonl 2>&1 || exit 1
timeout -k 10 240 python -u $E > gpurun_out/r6a_eg2m_$i.jsonl 2>&1 || exit 1
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $E > gpurun_out/r6a_eg4k_$i.jsonl 2>&1 || exit 1
done
