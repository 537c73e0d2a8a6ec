# A/B: ingress verdict kernel, qword lanes (product) vs the r1g dword lanes
set -e
O=gpurun_out/ingress_ab
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_ingress.py tests/test_rx_ring.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  LNX_PROF_INGRESS_UNROLL=1 timeout -k 10 120 python -u bench.py --op ingress --no-cpu-baseline --steps 100 > $O/bench_nopf_$i.jsonl 2>> $O/bench.err
  timeout -k 10 120 python -u bench.py --op ingress --no-cpu-baseline --steps 100 > $O/bench_pf_$i.jsonl 2>> $O/bench.err
done
echo done
