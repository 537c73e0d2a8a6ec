# r2d: lean rows with default-policy edge lines (variant 90) against the product: parity, A/B
set -e
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py mtu1500 0,90,53,91 11 > $O/var_mtu1500.log 2>&1
echo done
