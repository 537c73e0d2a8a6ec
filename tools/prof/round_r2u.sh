# r2u: rocprofv3 kernel trace of the r2 CRC32Search kernel (two captures per wave)
set -e
O=gpurun_out/r2u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/search_trace -o trace --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 20 --warmup 3 --prewarm-s 0.2 > $O/search_trace.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/search_pmc -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 5 --warmup 1 --prewarm-s 0 > $O/search_pmc.log 2>&1
echo done
