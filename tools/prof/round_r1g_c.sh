# r1g: lean line rows after the early-clobber fix — parity, debug check, timing
set -e
mkdir -p gpurun_out/r1g
timeout -k 10 400 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r1g/variants_parity_c.log 2>&1
timeout -k 10 200 python -u tools/debug/dbg_lean.py mtu1500 52 > gpurun_out/r1g/dbg52_c.txt 2>&1
timeout -k 10 200 python -u tools/prof/variants.py mtu1500 0,17,50,51,52,53,54 5 > gpurun_out/r1g/variants_mtu1500_c.txt 2>&1
timeout -k 10 200 python -u tools/prof/variants.py zipf64_1500 0,50 3 > gpurun_out/r1g/variants_zipf_c.txt 2>&1
