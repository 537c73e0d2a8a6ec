# r2zd: product with run-predicated narrow-row loads (NSR4 = 2): every GPU test, Zipf / 1500 B variants, Zipf bench line
set -e
O=gpurun_out/r2zd
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py zipf64_1500 0,125,122,124,26,0 5 > $O/var_zipf.log 2>&1
timeout -k 10 200 python -u bench.py --workload zipf64_1500 --no-cpu-baseline --verify > $O/bench_zipf64_1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --verify > $O/bench_mtu1500.jsonl 2>> $O/bench.err
echo done
