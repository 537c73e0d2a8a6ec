# r2c: tail balancing (work stealing between lean workgroups): parity incl. the forced-steal variant, A/B, timelines, bench
set -e
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -u tools/prof/variants.py mtu1500 0,7,59 9 > $O/var_mtu1500.log 2>&1
timeout -k 10 200 python -u tools/prof/timeline.py mtu1500 0 59 > $O/timeline_mtu1500.txt 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
echo done
