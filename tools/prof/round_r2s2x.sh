# r2s2x: last check of the committed tree: every GPU parity test, smoke, the default bench line
set -e
O=gpurun_out/r2s2x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_mtu1500.jsonl 2> $O/bench.err
echo done
