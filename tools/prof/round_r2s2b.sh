# r2s2b: CRC32Search pass B by word checks (four compares against Z_{-k}(residue) per word, one Z_4 step) against the
# r2 byte-chain pass B (LNX_PROF_SEARCH=b); '0' / '4' / '8' put 0 / 4 / 8 of pass B's Z_4 steps through the shared tables
set -e
O=gpurun_out/r2s2b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in b x 0 4 8; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
for z in b x; do
LNX_PROF_SEARCH=$z timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_$z -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_$z.log 2>&1
done
echo done
