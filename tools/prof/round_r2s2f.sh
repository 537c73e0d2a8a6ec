# r2s2f: CRC32Search U layout with two captures per half-wave (crc32_search_u_kernel<2>, the product now: two
# independent Z_4 chains per lane) against one per half ('u') and the two-block shared-table form ('x')
set -e
O=gpurun_out/r2s2f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p u x; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
LNX_PROF_SEARCH=p timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_p -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_p.log 2>&1
echo done
