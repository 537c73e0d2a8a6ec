# r2s2t: checkpoint after the CRC32Search group-descriptor loads: every GPU parity test, smoke, the search bench line
# with its CPU baseline, a rocprofv3 kernel trace of it, the headline bench line
set -e
O=gpurun_out/r2s2t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py --op search --verify > $O/bench_search_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_search -o trace --output-format csv -- python3 bench.py --op search --no-cpu-baseline --prewarm-s 0.2 --steps 20 --warmup 3 > $O/bench_trace_search.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2>> $O/bench.err
echo done
