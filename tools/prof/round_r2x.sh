# r2x: CRC32Search with 1, 2 or 4 interleaved copies of the Z_4 tables (LNX_PROF_SEARCH_ZREP), plus bank-conflict counters
set -e
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in 1 2 4; do
LNX_PROF_SEARCH_ZREP=$z timeout -k 10 200 python -u $B --verify > $O/zrep${z}_$r.jsonl 2>> $O/bench.err
done
done
for z in 1 4; do
LNX_PROF_SEARCH_ZREP=$z timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_$z -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_$z.log 2>&1
done
echo done
