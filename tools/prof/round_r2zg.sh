# r2zg: product with narrow-row load runs of 4 steps: every GPU test, bench lines, rocprofv3 profile of the Zipf mix
set -e
O=gpurun_out/r2zg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -u bench.py --workload zipf64_1500 --no-cpu-baseline --verify > $O/bench_zipf64_1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --verify > $O/bench_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op fcs_verify --no-cpu-baseline --verify > $O/bench_fcs_verify_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 900 bash tools/prof/profile.sh r2zg zipf64_1500 > $O/profile_zipf.log 2>&1
echo done
