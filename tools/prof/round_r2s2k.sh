# r2s2k: end-of-session checkpoint: every GPU parity test, smoke, a bench line per workload / op (verified on a
# sample), PMC counters of the ingress-verdict kernel against sum16 (the 0.75 vs 0.86 gap)
set -e
O=gpurun_out/r2s2k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 200 python -u bench.py > $O/bench_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --workload jumbo9000 --no-cpu-baseline --verify > $O/bench_jumbo9000.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --workload zipf64_1500 --no-cpu-baseline --verify > $O/bench_zipf64_1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op fcs_verify --no-cpu-baseline --verify > $O/bench_fcs_verify_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op sum16 --no-cpu-baseline --verify > $O/bench_sum16_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op ingress --no-cpu-baseline --verify > $O/bench_ingress_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op search --verify > $O/bench_search_mtu1500.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --op rx_ring --no-cpu-baseline > $O/bench_rx_ring.jsonl 2>> $O/bench.err
timeout -k 10 200 python -u bench.py --with-copies --no-cpu-baseline > $O/bench_with_copies_mtu1500.jsonl 2>> $O/bench.err
for op in ingress sum16; do
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc1_$op -o pmc --output-format csv -- python3 bench.py --op $op --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc1_$op.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc2_$op -o pmc --output-format csv -- python3 bench.py --op $op --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc2_$op.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc3_$op -o pmc --output-format csv -- python3 bench.py --op $op --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc3_$op.log 2>&1
done
echo done
