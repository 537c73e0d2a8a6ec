# r2v: CRC32Search pass A through lane-private nibble tables (NIB) against the shared Z_4 byte tables (ZWORDS=12)
set -e
O=gpurun_out/r2v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
timeout -k 10 200 python -u $B --verify > $O/nib_$r.jsonl 2>> $O/bench.err
LNX_PROF_SEARCH_ZWORDS=12 timeout -k 10 200 python -u $B --verify > $O/z4_$r.jsonl 2>> $O/bench.err
done
echo done
