# r2a: parity after the ADVICE r1 fixes (ring depth, IPv6 TCP verdicts, batch argument checks), smoke, bench line
set -e
O=gpurun_out/r2a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
echo done
