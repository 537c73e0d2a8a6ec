# r2ck: round-2 checkpoint after the search and edge-policy changes: every GPU parity test, smoke, and a bench line per workload / op
set -e
O=gpurun_out/r2ck
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --workload jumbo9000 --no-cpu-baseline --verify > $O/bench_jumbo9000.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --workload zipf64_1500 --no-cpu-baseline --verify > $O/bench_zipf64_1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op fcs_verify --no-cpu-baseline --verify > $O/bench_fcs_verify_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op sum16 --no-cpu-baseline --verify > $O/bench_sum16_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op ingress --no-cpu-baseline --verify > $O/bench_ingress_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op search --no-cpu-baseline --verify > $O/bench_search_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op rx_ring --no-cpu-baseline > $O/bench_rx_ring.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --with-copies --no-cpu-baseline > $O/bench_with_copies_mtu1500.jsonl 2>> $O/bench.err
echo done
