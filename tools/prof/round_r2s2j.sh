# r2s2j: PMC counters of the ingress-verdict kernel against sum16 on the same 1 M x 1500-B frames (where does the
# 0.75 vs 0.86 gap go), plus a grid sweep of the ingress kernel (workgroups per CU)
set -e
O=gpurun_out/r2s2j
mkdir -p $O
export TMPDIR=/tmp
for op in ingress sum16; do
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc1_$op -o pmc --output-format csv -- python3 bench.py --op $op --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc1_$op.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc2_$op -o pmc --output-format csv -- python3 bench.py --op $op --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc2_$op.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc3_$op -o pmc --output-format csv -- python3 bench.py --op $op --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc3_$op.log 2>&1
done
for w in 64 128 192; do
LNX_PROF_INGRESS_WG_PER_CU=$w timeout -k 10 200 python -u bench.py --op ingress --no-cpu-baseline --steps 100 > $O/ingress_wg$w.jsonl 2>> $O/bench.err
done
echo done
