# r2q: jumbo frames on two-word 16-lane rows with edge-line policy (variants 29 = 24-line items, 43 = 32, 44 = 18) against the 32-lane product (0)
set -e
O=gpurun_out/r2q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py jumbo9000 0,29,43,44 7 > $O/var_jumbo.log 2>&1
echo done
