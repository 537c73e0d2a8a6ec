# r2f: sum16 line rows with default-policy edge lines: parity, variants A/B, bench line
set -e
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/sum16_variants.py 9 0,5,2 > $O/sum16_variants.log 2>&1
timeout -k 10 200 python -u bench.py --op sum16 --verify --no-cpu-baseline > $O/bench_sum16_mtu1500.jsonl 2> $O/bench.err
echo done
