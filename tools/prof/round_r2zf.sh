# r2zf: narrow-row load runs NSR 2 (product, 0) / 4 (122) / 6 (126) , 10 interleaved reps, two processes; parity of 126/127
set -e
O=gpurun_out/r2zf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -x -q --timeout 120 --timeout-method thread -k "126" > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py zipf64_1500 0,122,126 10 > $O/var_zipf_1.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py zipf64_1500 126,122,0 10 > $O/var_zipf_2.log 2>&1
echo done
