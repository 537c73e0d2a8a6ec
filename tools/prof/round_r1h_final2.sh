# r1h final 2: parity, smoke, default bench line, search line + kernel-trace --stats
set -e
O=gpurun_out/r1h_final2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --op search --verify --no-cpu-baseline > $O/bench_search_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/search_trace -o trace --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 20 --warmup 3 --prewarm-s 0.2 > $O/search_trace.log 2>&1
echo done
