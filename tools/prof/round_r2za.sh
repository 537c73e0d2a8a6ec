# r2za: sorted 4-lane rows (sorted_body) on the Zipf mix: parity of the new variants, then A/B against the product
# (r2za_1: one item per wave in flight; r2za_2: next window's bounds prefetched; this run: two items in flight, compiler-visible loads)
# (the sorted-row variants 110-114 were removed after these runs; profiles/r2zab_zipf_sorted_rows_rejected.txt)
set -e
O=gpurun_out/r2za
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py -x -v --timeout 120 --timeout-method thread -k "110 or 112 or 113 or 114" > $O/gpu_tests.log 2>&1
for v in 0 110 111 114 112 26; do
timeout -k 10 120 python -u tools/prof/variants.py zipf64_1500 $v 5 >> $O/var_zipf.log 2>&1
done
echo done
