# r2y: CRC32Search with lane-private Z_4 tables (LNX_PROF_SEARCH_ZWORDS=99, one workgroup per CU; second run: two chains per lane) against the product
set -e
O=gpurun_out/r2y
mkdir -p $O
LNX_PROF_SEARCH_ZWORDS=99 timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
LNX_PROF_SEARCH_ZWORDS=99 timeout -k 10 200 python -u $B --verify > $O/priv_$r.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u $B --verify > $O/prod_$r.jsonl 2>> $O/bench.err
done
LNX_PROF_SEARCH_ZWORDS=99 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_priv -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_priv.log 2>&1
echo done
