set -e
mkdir -p gpurun_out/r2k
timeout -k 10 400 python -u tools/prof/variants.py zipf64_1500 0,22,17,21,18,19,50,10,26,27 5 > gpurun_out/r2k/var_zipf.log 2>&1
echo done
