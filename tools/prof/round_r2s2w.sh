# r2s2w: CRC32Search with the next group's bounds loaded one iteration ahead ('B') against the product ('p'); then
# every GPU parity test on the final tree
set -e
O=gpurun_out/r2s2w
mkdir -p $O
export TMPDIR=/tmp
LNX_PROF_SEARCH=B timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_B.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p B; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
echo done
