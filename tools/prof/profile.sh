#!/bin/bash
# Profile bench.py's CRC kernel with rocprofv3 on the GPU box.
#   tools/prof/profile.sh TAG [bench args...]
# Writes gpurun_out/prof_TAG/: kernel-trace stats (timing pass) and separate
# PMC passes (one counter group per pass; never combined with tracing domains).
set -u
TAG=${1:-run}; shift || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
ARGS="--steps 20 --warmup 3 --no-cpu-baseline $*"
echo "[prof] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
for grp in "$@"; do :; done
i=0
for CNT in "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "[prof] pmc pass $i: $CNT"
  timeout -k 10 300 rocprofv3 --pmc $CNT -d $OUT/pmc$i -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $* > $OUT/bench_pmc$i.log 2>&1 || echo "pmc pass $i failed rc=$?"
done
echo "[prof] done"
