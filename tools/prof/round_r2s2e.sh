# r2s2e: CRC32Search with every Z_4 step of pass A and of the word-check pass B through the lane-private U layout
# (crc32_search_u_kernel, one 16-wave block per CU, the product now) against the r2s2d form ('x', shared Z_4 in pass A,
# byte chains in pass B, 2 blocks per CU) and the r2 product ('b')
set -e
O=gpurun_out/r2s2e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in u x b; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
LNX_PROF_SEARCH=u timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_u -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_u.log 2>&1
echo done
