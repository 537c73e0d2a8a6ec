# PMC passes over the staged lane streams (research variants) and the product
# on one workload: tools/prof/variants.py times each variant, rocprofv3 counts
# per dispatch (one counter group per pass, never with tracing).
#   bash tools/prof/stage_pmc.sh TAG WORKLOAD VARIANTS   (VARIANTS as 0+302)
set -u
TAG=${1:-stage_pmc}
WL=${2:-zipf64_1500}
VS=${3:-0+302}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
i=0
for CNT in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" \
           "FETCH_SIZE TCC_REQ_sum"; do
  i=$((i+1))
  echo "[stage_pmc] pass $i: $CNT"
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d $O/pmc$i -o pmc --output-format csv -- python3 tools/prof/variants.py $WL $VS 1 > $O/pmc$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $O/pmc$i.log; exit 1; }
done
python3 tools/prof/pmc_table.py $O > $O/table.txt && cat $O/table.txt
