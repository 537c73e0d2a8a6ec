#!/bin/bash
# One gpurun session: the named steps in order, each under its own time limit,
# stopping at the first failure (a GPU step that faults or times out ends the
# session; nothing is retried).  Output under gpurun_out/TAG/.
#
#   tools/prof/gpu_session.sh TAG STEP [STEP ...]
#
# Steps:
#   tests[:EXPR]      pytest -m gpu (optionally -k EXPR; "_or_" stands for " or ")
#   smoke             __graft_entry__.smoke()
#   bench             the default bench line (what the driver runs)
#   lines             a --verify'd bench line per workload / op
#   line:WL:OP[:ARGS] one bench line (ARGS: extra flags, comma-separated)
#   prof:WL[:OP[:short]] rocprofv3 kernel trace + PMC passes (tools/prof/profile.sh)
#   py:FILE[:ARGS]    python FILE (a measurement script), ARGS comma-separated
#   sh:FILE[:ARGS]    bash FILE (a measurement script), ARGS comma-separated
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {  # run LIMIT LOG CMD...: one step, its own time limit
  local lim=$1 log=$2; shift 2
  echo "[$TAG] $(date +%T) $*"
  timeout -k 10 $lim "$@" >> $log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[$TAG] step failed rc=$rc: $*"; tail -20 $log; exit $rc; fi
}
for STEP in "$@"; do
  IFS=: read -r KIND A B C <<< "$STEP"
  case $KIND in
    tests)
      if [ -n "$A" ]; then
        run 900 $O/gpu_tests.log python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${A//_or_/ or }"
      else
        run 900 $O/gpu_tests.log python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
      fi
      tail -3 $O/gpu_tests.log ;;
    smoke) run 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 240 $O/bench_default.jsonl python -u bench.py --steps 20 --warmup 5; tail -1 $O/bench_default.jsonl ;;
    lines)
      run 240 $O/bench_mtu1500.jsonl python -u bench.py --verify
      for WL in jumbo9000 zipf64_1500; do
        run 240 $O/bench_$WL.jsonl python -u bench.py --workload $WL --no-cpu-baseline --verify
      done
      for OP in fcs_verify sum16 ingress search fcs_append tx_checksum; do
        run 240 $O/bench_${OP}_mtu1500.jsonl python -u bench.py --op $OP --no-cpu-baseline --verify
      done
      run 240 $O/bench_with_copies_mtu1500.jsonl python -u bench.py --with-copies --no-cpu-baseline ;;
    line)
      EXTRA=${C//,/ }
      run 300 $O/bench_${A}_${B}.jsonl python -u bench.py --workload $A --op $B $EXTRA
      tail -1 $O/bench_${A}_${B}.jsonl ;;
    prof) run 900 $O/prof_${A}_${B:-crc32}.log bash tools/prof/profile.sh $TAG $A ${B:-crc32} $C ;;
    py)  # a python script, or an executable (a microbenchmark binary built in-tree)
      if [[ $A == *.py ]]; then run 600 $O/py_$(basename $A .py).log python -u $A ${B//,/ };
      else run 600 $O/py_$(basename $A).log ./$A ${B//,/ }; fi
      tail -30 $O/py_$(basename $A .py).log ;;
    sh) run 600 $O/sh_$(basename $A .sh).log bash $A ${B//,/ }; tail -30 $O/sh_$(basename $A .sh).log ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
echo "[$TAG] $(date +%T) done"
