# r2ze: narrow-row load runs NSR 2 (product, 0) / 4 (122) / none (125), 10 interleaved reps, two processes
set -e
O=gpurun_out/r2ze
mkdir -p $O
timeout -k 10 300 python -u tools/prof/variants.py zipf64_1500 0,122,125 10 > $O/var_zipf_1.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py zipf64_1500 125,122,0 10 > $O/var_zipf_2.log 2>&1
echo done
