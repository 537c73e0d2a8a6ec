# r2b: lean rows with the frame-end junk bytes masked in the fold (no reload): parity, then A/B
set -e
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -u tools/prof/variants.py mtu1500 0,57,53,58 9 > $O/var_mtu1500.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
echo done
