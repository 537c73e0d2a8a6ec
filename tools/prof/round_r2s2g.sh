# r2s2g: CRC32Search U layout with the next capture group prefetched (bounds one iteration ahead, first-block words
# issued before pass B): one capture per half ('1'), two per half ('q', spills 144 B), against the product ('p', two
# per half, no prefetch)
set -e
O=gpurun_out/r2s2g
mkdir -p $O
LNX_PROF_SEARCH=1 timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_1.log 2>&1
LNX_PROF_SEARCH=q timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_q.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p 1 q; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
echo done
