#!/bin/bash
# Profile bench.py's CRC kernel with rocprofv3 on the GPU box.
#   tools/prof/profile.sh TAG WORKLOAD
# Writes gpurun_out/prof_TAG_WORKLOAD/: a kernel-trace --stats pass (timing) and
# separate PMC passes (one counter group each, never combined with tracing),
# plus a FETCH_SIZE pass over tools/prof/calib (known byte counts).
set -u
TAG=${1:-run}
WL=${2:-mtu1500}
OUT=gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --workload $WL --no-cpu-baseline"
BT="$B --prewarm-s 0.2"
B="$B --prewarm-s 0"
echo "[prof] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $BT --steps 20 --warmup 3 > $OUT/bench_trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
i=0
for CNT in "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "[prof] pmc pass $i: $CNT"
  timeout -k 10 300 rocprofv3 --pmc $CNT -d $OUT/pmc$i -o pmc --output-format csv -- python3 $B --steps 5 --warmup 1 > $OUT/bench_pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
done
echo "[prof] calibration"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o calib --output-format csv -- tools/prof/calib > $OUT/calib.log 2>&1 || { echo "calib failed rc=$?"; exit 1; }
echo "[prof] done"
