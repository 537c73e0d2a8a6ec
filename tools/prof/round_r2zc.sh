# r2zc: 4-lane rows loading only the runs of steps their item has (variants 120-124) against the product on the Zipf mix
set -e
O=gpurun_out/r2zc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -x -v --timeout 120 --timeout-method thread -k "120 or 122 or 123 or 124" > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u tools/prof/variants.py zipf64_1500 0,120,121,122,124,26,0 5 > $O/var_zipf.log 2>&1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o pmc --output-format csv -- python3 tools/prof/variants.py zipf64_1500 0,120,121,26 1 > $O/pmc.log 2>&1
echo done
