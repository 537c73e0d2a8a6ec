# r1g: lean line rows — parity of the forced variants, then timing and PMC
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread -k "50 or 51 or 52 or 17 or 18" > gpurun_out/r1g/variants_parity.log 2>&1
timeout -k 10 200 python -u tools/prof/variants.py mtu1500 0,17,18,50,51,52,53,54 5 > gpurun_out/r1g/variants_mtu1500.txt 2>&1
timeout -k 10 200 python -u tools/prof/variants.py jumbo9000 0,50 3 > gpurun_out/r1g/variants_jumbo9000.txt 2>&1
bash tools/prof/pmc_variants.sh r1g_lean mtu1500 0,50,53,54
