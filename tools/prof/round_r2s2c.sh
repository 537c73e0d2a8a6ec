# r2s2c: word-check CRC32Search pass B with byte-chain Z_4 steps ('0') by pass A split (LNX_PROF_SEARCH_ZWORDS: words of
# pass A through the shared Z_4 tables, the rest by the conflict-free byte column), the lane-private nibble Z_4 form ('n'),
# and the r2 product ('b')
set -e
O=gpurun_out/r2s2c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
LNX_PROF_SEARCH=0 LNX_PROF_SEARCH_ZWORDS=8 timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_0_8.log 2>&1
LNX_PROF_SEARCH=n timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_n.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
LNX_PROF_SEARCH=b timeout -k 10 200 python -u $B --verify > $O/mode_b_$r.jsonl 2>> $O/bench.err
LNX_PROF_SEARCH=n timeout -k 10 200 python -u $B --verify > $O/mode_n_$r.jsonl 2>> $O/bench.err
for z in 12 10 8 6 4; do
LNX_PROF_SEARCH=0 LNX_PROF_SEARCH_ZWORDS=$z timeout -k 10 200 python -u $B --verify > $O/mode_0_z${z}_$r.jsonl 2>> $O/bench.err
done
done
for z in 0 n; do
LNX_PROF_SEARCH=$z timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_$z -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_$z.log 2>&1
done
echo done
