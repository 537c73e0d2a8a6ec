# r1g: product with lean line rows below 1600 B mean — tests, dispatch tuning, bench
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g/gpu_tests_e.log 2>&1
timeout -k 10 100 python -u tools/prof/variants.py mtu1500 0,56,50 5 > gpurun_out/r1g/tune_e.txt 2>&1
timeout -k 10 100 python -u tools/prof/variants.py uni640_1536 0,56 3 >> gpurun_out/r1g/tune_e.txt 2>&1
timeout -k 10 100 python -u tools/prof/variants.py fixed1024 0,56 3 >> gpurun_out/r1g/tune_e.txt 2>&1
timeout -k 10 100 python -u tools/prof/variants.py fixed2048 0,55,51 3 >> gpurun_out/r1g/tune_e.txt 2>&1
timeout -k 10 100 python -u tools/prof/variants.py fixed3072 0,55 3 >> gpurun_out/r1g/tune_e.txt 2>&1
timeout -k 10 200 python -u bench.py > gpurun_out/r1g/bench_mtu1500_e.jsonl 2> gpurun_out/r1g/bench_mtu1500_e.err
