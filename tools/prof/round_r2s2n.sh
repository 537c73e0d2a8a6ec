# r2s2n: CRC32Search with global loads and the next capture group prefetched ('f': one capture per half, 'F': two,
# spills 144 B) against the product ('p')
set -e
O=gpurun_out/r2s2n
mkdir -p $O
export TMPDIR=/tmp
LNX_PROF_SEARCH=f timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_f.log 2>&1
LNX_PROF_SEARCH=F timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_F.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p f F; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
echo done
