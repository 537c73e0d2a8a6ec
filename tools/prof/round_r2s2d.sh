# r2s2d: CRC32Search after the VALU trims (pass A Z_4 steps fused into v_bitop3 with the next word, pass B byte
# chains on the pre-XOR-ed word, hit ballots straight from the compares, 32-bit candidate bounds): product (word checks,
# byte-chain steps) against the r2 byte-chain pass B ('b'), 4 of 11 steps by shared Z_4 ('4'), all shared ('z'), nibble ('n')
set -e
O=gpurun_out/r2s2d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
LNX_PROF_SEARCH=4 timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_4.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in x b 4 z n; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
LNX_PROF_SEARCH=x timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_x -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_x.log 2>&1
LNX_PROF_SEARCH=x timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $O/pmc2_x -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc2_x.log 2>&1
echo done
