# r2s2h: CRC32Search segments as two 24-byte chains joined by Z_24 ('1': one capture per half, 'q': two) against the
# product ('p'); then the checkpoint after the CRC32Search rework: every GPU parity test, smoke, the search bench line
# (with its CPU baseline), a rocprofv3 kernel trace of the search bench, the headline bench line
set -e
O=gpurun_out/r2s2h
mkdir -p $O
export TMPDIR=/tmp
LNX_PROF_SEARCH=1 timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_1.log 2>&1
LNX_PROF_SEARCH=q timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_q.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p 1 q; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py --op search --verify > $O/bench_search_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_search -o trace --output-format csv -- python3 bench.py --op search --no-cpu-baseline --prewarm-s 0.2 --steps 20 --warmup 3 > $O/bench_trace_search.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2>> $O/bench.err
echo done
