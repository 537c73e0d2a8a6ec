# r2z: 4-lane rows with three or four slots in flight on the Zipf mix (variants 66-69) against the product
set -e
mkdir -p gpurun_out/r2z
timeout -k 10 400 python -u tools/prof/variants.py zipf64_1500 0,65,66,67,68,69,0 5 > gpurun_out/r2z/var_zipf.log 2>&1
echo done
