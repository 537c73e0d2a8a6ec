# r2s2i: CRC32Search with 16-byte loads where the four dwords hold capture bytes ('v'; 'W' with split chains)
# against the product ('p': one dword per lane per load instruction, ~13 touches per 128-byte line)
set -e
O=gpurun_out/r2s2i
mkdir -p $O
export TMPDIR=/tmp
LNX_PROF_SEARCH=v timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_v.log 2>&1
LNX_PROF_SEARCH=W timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_W.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p v W; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
for z in p v; do
LNX_PROF_SEARCH=$z timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $O/pmc_$z -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_$z.log 2>&1
done
echo done
