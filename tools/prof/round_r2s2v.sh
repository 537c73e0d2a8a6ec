# r2s2v: final checkpoint of the session's tree: every GPU parity test, smoke, a bench line per workload / op
set -e
O=gpurun_out/r2s2v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --workload jumbo9000 --no-cpu-baseline --verify > $O/bench_jumbo9000.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --workload zipf64_1500 --no-cpu-baseline --verify > $O/bench_zipf64_1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op fcs_verify --no-cpu-baseline --verify > $O/bench_fcs_verify_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op sum16 --no-cpu-baseline --verify > $O/bench_sum16_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op ingress --no-cpu-baseline --verify > $O/bench_ingress_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op search --verify > $O/bench_search_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op fcs_append --verify > $O/bench_fcs_append_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --with-copies --no-cpu-baseline > $O/bench_with_copies_mtu1500.jsonl 2>> $O/bench.err
echo done
