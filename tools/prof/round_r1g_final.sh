# r1g final: parity, smoke, bench lines for configs[1..3] and ops, rocprofv3 profiles of the product
set -e
mkdir -p gpurun_out/r1g_final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g_final/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1g_final/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > gpurun_out/r1g_final/bench_mtu1500.jsonl 2> gpurun_out/r1g_final/bench.err
timeout -k 10 200 python -u bench.py --workload jumbo9000 > gpurun_out/r1g_final/bench_jumbo9000.jsonl 2>> gpurun_out/r1g_final/bench.err
timeout -k 10 200 python -u bench.py --workload zipf64_1500 > gpurun_out/r1g_final/bench_zipf64_1500.jsonl 2>> gpurun_out/r1g_final/bench.err
timeout -k 10 200 python -u bench.py --op fcs_verify --no-cpu-baseline > gpurun_out/r1g_final/bench_fcs_verify_mtu1500.jsonl 2>> gpurun_out/r1g_final/bench.err
timeout -k 10 200 python -u bench.py --op sum16 --no-cpu-baseline > gpurun_out/r1g_final/bench_sum16_mtu1500.jsonl 2>> gpurun_out/r1g_final/bench.err
bash tools/prof/profile.sh r1g_final mtu1500 > gpurun_out/r1g_final/prof_mtu1500.log 2>&1
bash tools/prof/profile.sh r1g_final jumbo9000 > gpurun_out/r1g_final/prof_jumbo9000.log 2>&1
