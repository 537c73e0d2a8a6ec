# r2n: CRC32Search with two captures per wave (48-byte segments, five-level scans): parity, A/B against the r1h kernel
set -e
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
LNX_PROF_SEARCH=s timeout -k 10 200 python -u $B --verify > $O/seg24.jsonl 2> $O/bench.err
for z in 8 10 12; do
LNX_PROF_SEARCH_ZWORDS=$z timeout -k 10 200 python -u $B --verify > $O/half_z$z.jsonl 2>> $O/bench.err
done
LNX_PROF_SEARCH=s timeout -k 10 200 python -u $B > $O/seg24_b.jsonl 2>> $O/bench.err
echo done
