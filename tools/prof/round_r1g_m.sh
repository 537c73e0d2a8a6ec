# r1g: lean rows with wave-uniform per-step branches (skip / unpredicated / predicated) and OOB load runs
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g/gpu_tests_m.log 2>&1
timeout -k 10 100 python -u tools/prof/variants.py mtu1500 0,56 5 > gpurun_out/r1g/tune_m.txt 2>&1
timeout -k 10 100 python -u tools/prof/variants.py uni640_1536 0,56 5 >> gpurun_out/r1g/tune_m.txt 2>&1
timeout -k 10 100 python -u tools/prof/variants.py fixed1024 0,56 5 >> gpurun_out/r1g/tune_m.txt 2>&1
timeout -k 10 100 python -u tools/prof/variants.py zipf64_1500 0,56 3 >> gpurun_out/r1g/tune_m.txt 2>&1
