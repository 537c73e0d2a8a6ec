# A/B of the search kernel's pass A (Z_4 words vs byte column) + LDS conflict counters
set -e
O=gpurun_out/search_ab
mkdir -p $O
# LNX_PROF_* knobs are read by the research library only
export LNETO_AMD_LIB=$PWD/lneto_amd/liblneto_amd_research.so
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for m in 3 2 1 0; do
  LNX_PROF_SEARCH=$m timeout -k 10 120 python -u bench.py --op search --verify --no-cpu-baseline --steps 100 > $O/bench_$m.jsonl 2>> $O/bench.err
  LNX_PROF_SEARCH=$m timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES -d $O/pmc_$m -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_$m.log 2>&1
done
echo done
