# r1g: lean rows with the last step out of range for 12-line frames
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g/gpu_tests_g.log 2>&1
timeout -k 10 100 python -u tools/prof/variants.py mtu1500 0,56,53 7 > gpurun_out/r1g/tune_g.txt 2>&1
timeout -k 10 200 python -u bench.py > gpurun_out/r1g/bench_mtu1500_g.jsonl 2> gpurun_out/r1g/bench_mtu1500_g.err
bash tools/prof/profile.sh r1g2 mtu1500 > gpurun_out/r1g/prof2_mtu1500.log 2>&1
