# r2zb: counters of the sorted 4-lane rows (110, loads only 111) against rows_body (0, loads only 26) on the Zipf mix
set -e
# (the sorted-row variants 110-114 were removed after these runs; profiles/r2zab_zipf_sorted_rows_rejected.txt)
export TMPDIR=/tmp
bash tools/prof/pmc_variants.sh r2zb zipf64_1500 0,110,111,26 > gpurun_out/r2zb_inst.log 2>&1
O=gpurun_out/pmcvar_r2zb_fetch
mkdir -p $O
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/pmc -o pmc --output-format csv -- python3 tools/prof/variants.py zipf64_1500 0,110,111,26 1 > $O/run.log 2>&1
echo done
