# Per-dispatch instruction counters for CRC kernel variants (one PMC pass, no tracing).
#   tools/prof/pmc_variants.sh TAG WORKLOAD V1+V2+... [C1+C2+... [SUFFIX]]
# (WORKLOAD append: tools/prof/append_ab.py's variants instead of variants.py's)
set -eu
TAG=$1; WL=$2; VARS=$3
CTRS=${4:-SQ_INSTS_VALU+SQ_INSTS_SALU+SQ_INSTS_LDS+SQ_INSTS_VMEM_RD}
OUT=gpurun_out/pmcvar_${TAG}_${WL}${5:+_$5}
mkdir -p $OUT
export TMPDIR=/tmp
# WORKLOAD "append": the TX append A/B script (its variants, m1 = no append)
if [ "$WL" = append ]; then SCRIPT=tools/prof/append_ab.py; ARGS="$VARS 1"; else SCRIPT=tools/prof/variants.py; ARGS="$WL $VARS 1"; fi
timeout -k 10 120 rocprofv3 --pmc ${CTRS//+/ } -d $OUT/pmc -o pmc --output-format csv -- python3 $SCRIPT $ARGS > $OUT/run.log 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
f = glob.glob(out + "/pmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "crc32_rows_kernel" not in k: continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(out + "/summary.txt", "w") as fo:
    for k, d in acc.items():
        args = k[k.find("<") + 1:k.find(">")]
        line = args + " | " + " ".join(f"{c}={sorted(v)[len(v)//2]:.4g}" for c, v in sorted(d.items()))
        print(line); fo.write(line + "\n")
PY
