# r2s2s: CRC32Search loads of packed capture groups through one buffer descriptor per group (one per-lane offset, the
# word in the immediate, no guards): merged into 16-byte loads by hipcc (product, 'p'), kept as dwords by alternating
# the nt bit ('G'), against the guarded global loads ('g')
set -e
O=gpurun_out/r2s2s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
LNX_PROF_SEARCH=G timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_G.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p G g; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
for z in p G g; do
LNX_PROF_SEARCH=$z timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS -d $O/pmc_$z -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_$z.log 2>&1
done
echo done
