# r1h final 3: parity, smoke, default bench line, sum16 and ingress lines at the new grids
set -e
O=gpurun_out/r1h_final3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --op sum16 --verify --no-cpu-baseline > $O/bench_sum16_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op ingress --verify --no-cpu-baseline > $O/bench_ingress_mtu1500.jsonl 2>> $O/bench.err
echo done
