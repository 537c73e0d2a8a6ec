#!/bin/bash
# Profile one bench.py kernel with rocprofv3 on the GPU box.
#   tools/prof/profile.sh TAG WORKLOAD [OP [short]]
# Writes gpurun_out/prof_TAG_WORKLOAD[_OP]/: a kernel-trace --stats pass
# (timing, with a bench line of its own) and separate PMC passes (one counter
# group each, never combined with tracing), plus a FETCH_SIZE pass over
# tools/prof/calib (known byte counts).  tools/prof/summarize.py turns it into
# profiles/.
set -u
TAG=${1:-run}
WL=${2:-mtu1500}
OP=${3:-crc32}
SHORT=${4:-}   # "short": the staged lane-stream entry (bench.py --short-frames)
SUF=$WL; [ "$OP" != crc32 ] && SUF=${WL}_$OP
XA=""; [ "$SHORT" = short ] && { SUF=${SUF}_short; XA="--short-frames"; }
OUT=gpurun_out/prof_${TAG}_${SUF}
mkdir -p $OUT
export TMPDIR=/tmp
# --no-slice16m: the N=1 mtu1500 line's 16 M-frame sub-measurement would land
# in the trace and the counter passes as launches of the same kernel
B="bench.py --workload $WL --op $OP --no-cpu-baseline --no-slice16m $XA"
BT="$B --prewarm-s 0.5"
B="$B --prewarm-s 0"
echo "[prof] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $BT --steps 50 --warmup 5 > $OUT/bench_trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
i=0
for CNT in "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY WRITE_SIZE"; do
  i=$((i+1))
  echo "[prof] pmc pass $i: $CNT"
  # (--kernel-trace beside the counters: the GRBM pass's per-dispatch clock,
  # summarize.py; that pass warms the GPU first so its clock is the steady one)
  BP="$B"; case "$CNT" in *GRBM*) BP="${B/--prewarm-s 0/--prewarm-s 0.5}";; esac
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace -d $OUT/pmc$i -o pmc --output-format csv -- python3 $BP --steps 5 --warmup 1 > $OUT/bench_pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
done
echo "[prof] calibration"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o calib --output-format csv -- tools/prof/calib > $OUT/calib.log 2>&1 || { echo "calib failed rc=$?"; exit 1; }
echo "[prof] done"
