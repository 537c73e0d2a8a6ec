set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l
timeout -k 10 300 python -u tools/prof/variants.py zipf64_1500 314,340,342 7 > gpurun_out/r5l/variants.log 2>&1 || exit 1
for V in 314 340 342; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/r5l/v$V -o v$V --output-format csv -- python3 tools/prof/zipf_diag.py $V > gpurun_out/r5l/v$V.log 2>&1 || { echo "pmc $V failed"; exit 1; }
done
echo done
