# r2e: lean rows with default-policy edge lines as the product: parity, policy A/B, bench
set -e
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py mtu1500 0,90,92,93,53,91 9 > $O/var_mtu1500.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --op fcs_verify --no-cpu-baseline > $O/bench_fcs_verify_mtu1500.jsonl 2>> $O/bench.err
echo done
