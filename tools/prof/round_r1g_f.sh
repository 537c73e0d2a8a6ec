# r1g: bench lines for configs[1..3] and rocprofv3 profiles of the lean-row product
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 200 python -u bench.py > gpurun_out/r1g/bench_mtu1500.jsonl 2> gpurun_out/r1g/bench_mtu1500.err
timeout -k 10 200 python -u bench.py --workload jumbo9000 > gpurun_out/r1g/bench_jumbo9000.jsonl 2> gpurun_out/r1g/bench_jumbo9000.err
timeout -k 10 200 python -u bench.py --workload zipf64_1500 > gpurun_out/r1g/bench_zipf64_1500.jsonl 2> gpurun_out/r1g/bench_zipf64_1500.err
bash tools/prof/profile.sh r1g mtu1500 > gpurun_out/r1g/prof_mtu1500.log 2>&1
bash tools/prof/profile.sh r1g jumbo9000 > gpurun_out/r1g/prof_jumbo9000.log 2>&1
bash tools/prof/profile.sh r1g zipf64_1500 > gpurun_out/r1g/prof_zipf64_1500.log 2>&1
