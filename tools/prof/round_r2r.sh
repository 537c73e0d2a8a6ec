# r2r: the >2 GiB generic-path test alone (timed)
set -e
O=gpurun_out/r2r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k generic -x -v --timeout 240 --timeout-method thread --durations=3 > $O/gpu_tests.log 2>&1
echo done
