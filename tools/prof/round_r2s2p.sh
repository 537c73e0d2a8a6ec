# r2s2p: segment mode (ring slots: lnx_crc32_segments, the TX FCS append, the receive ring's FCS verify) on the lean
# line rows: every GPU parity test, the FCS append and receive-ring bench lines, a kernel trace of the FCS append
set -e
O=gpurun_out/r2s2p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -u bench.py --op fcs_append --verify > $O/bench_fcs_append_mtu1500.jsonl 2> $O/bench.err
timeout -k 10 200 python -u bench.py --op rx_ring --no-cpu-baseline > $O/bench_rx_ring.jsonl 2>> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- python3 bench.py --op fcs_append --prewarm-s 0.2 --steps 20 --warmup 3 > $O/bench_trace.log 2>&1
echo done
