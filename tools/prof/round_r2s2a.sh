# r2s2a: lane-stream read ceiling (tools/ubench/lanestream.hip), then re-entry check of the restored tree: every GPU parity test, smoke, default bench line, Zipf line
set -e
O=gpurun_out/r2s2a
mkdir -p $O
timeout -k 10 120 ./tools/ubench/lanestream > $O/lanestream.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --workload zipf64_1500 --no-cpu-baseline --verify > $O/bench_zipf64_1500.jsonl 2>> $O/bench.err
echo done
