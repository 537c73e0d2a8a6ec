# r2s2o: bench line for the TX FCS append (lnx_fcs_append_batch over 1 M x 1496-B frames in 1536-B slots, verified on
# a sample), and a rocprofv3 kernel trace of it (its three launches plus the length reset)
set -e
O=gpurun_out/r2s2o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --op fcs_append --verify > $O/bench_fcs_append_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --op fcs_append --prewarm-s 0.2 --steps 20 --warmup 3 > $O/bench_trace.log 2>&1
echo done
