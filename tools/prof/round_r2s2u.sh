# r2s2u: ingress verdicts with the first batch loaded through one buffer descriptor per wave group: parity, bench
# lines, VALU counter
set -e
O=gpurun_out/r2s2u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ingress.py tests/test_rx_ring.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
for r in 1 2; do
timeout -k 10 200 python -u bench.py --op ingress --no-cpu-baseline --verify > $O/bench_ingress_$r.jsonl 2>> $O/bench.err
done
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc1_ingress -o pmc --output-format csv -- python3 bench.py --op ingress --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc1_ingress.log 2>&1
echo done
