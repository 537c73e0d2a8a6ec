# r2t: CRC32Search parity (incl. the two-captures-per-wave pairing test)
set -e
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
echo done
