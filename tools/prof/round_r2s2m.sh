# r2s2m: CRC32Search loads as global_load instead of flat_load (flat loads also count in lgkmcnt, so every wait for
# an LDS lookup waited for them): parity tests, product and the two-block form ('x')
set -e
O=gpurun_out/r2s2m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_search.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
B="bench.py --op search --no-cpu-baseline --steps 50"
for r in 1 2; do
for z in p x; do
LNX_PROF_SEARCH=$z timeout -k 10 200 python -u $B --verify > $O/mode_${z}_$r.jsonl 2>> $O/bench.err
done
done
echo done
