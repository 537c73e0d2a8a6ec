# r2i: 32-lane line rows (jumbo) with default-policy edge lines: parity, A/B, bench line
set -e
O=gpurun_out/r2i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py jumbo9000 0,97 9 > $O/var_jumbo9000.log 2>&1
timeout -k 10 200 python -u bench.py --workload jumbo9000 --no-cpu-baseline > $O/bench_jumbo9000.jsonl 2> $O/bench.err
echo done
