# r1g GPU session (restored container): parity tests, smoke, default bench line
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1g/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > gpurun_out/r1g/bench_mtu1500.jsonl 2> gpurun_out/r1g/bench_mtu1500.err
