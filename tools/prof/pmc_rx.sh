# PMC passes for one bench.py op (no trace): tools/prof/pmc_rx.sh TAG OP [WORKLOAD]
set -u
TAG=$1; OP=$2; WL=${3:-mtu1500}
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --workload $WL --op $OP --no-cpu-baseline --no-slice16m --prewarm-s 0 --steps 5 --warmup 1"
i=0
for CNT in "FETCH_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_MISC" "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT -d $OUT/pmc$i -o pmc --output-format csv -- python3 $B > $OUT/bench_pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; exit 1; }
done
echo done
