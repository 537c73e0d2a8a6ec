# r1g: lean rows with perm-addressed F pairs and deferred claims
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g/gpu_tests_d.log 2>&1
timeout -k 10 200 python -u tools/prof/variants.py mtu1500 0,17,50,51,53,54 5 > gpurun_out/r1g/variants_mtu1500_d.txt 2>&1
bash tools/prof/pmc_variants.sh r1g_d mtu1500 0,50
