# r1f GPU session: parity tests, bench lines for configs[1..3], rocprof for 1500 B and 9000 B
set -e
mkdir -p gpurun_out/r1f
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1f/gpu_tests.log 2>&1
timeout -k 10 200 python -u bench.py > gpurun_out/r1f/bench_mtu1500.jsonl 2> gpurun_out/r1f/bench_mtu1500.err
timeout -k 10 200 python -u bench.py --workload jumbo9000 > gpurun_out/r1f/bench_jumbo9000.jsonl 2> gpurun_out/r1f/bench_jumbo9000.err
timeout -k 10 200 python -u bench.py --workload zipf64_1500 > gpurun_out/r1f/bench_zipf64_1500.jsonl 2> gpurun_out/r1f/bench_zipf64_1500.err
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1f/smoke.log 2>&1
bash tools/prof/profile.sh r1f mtu1500 > gpurun_out/r1f/prof_mtu1500.log 2>&1
bash tools/prof/profile.sh r1f jumbo9000 > gpurun_out/r1f/prof_jumbo9000.log 2>&1
