# A/B of search kernel forms (LNX_PROF_SEARCH modes of the research library):
# per mode, the GPU search tests, a --verify'd bench line and one PMC pass of
# LDS bank conflicts / LDS-active / VALU / busy cycles.  Mode "p" is the
# product form (the research library's default branch).
#   bash tools/prof/search_ab.sh TAG MODE [MODE ...]
set -e
TAG=${1:-search_ab}; shift
O=gpurun_out/$TAG
mkdir -p $O
# LNX_PROF_* knobs are read by the research library only
export LNETO_AMD_LIB=$PWD/lneto_amd/liblneto_amd_research.so
export TMPDIR=/tmp
for m in "$@"; do
  mm=$m; [ "$m" = p ] && mm=
  LNX_PROF_SEARCH=$mm timeout -k 10 200 python -u -m pytest tests/test_search.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$m.log 2>&1
  tail -1 $O/tests_$m.log
  LNX_PROF_SEARCH=$mm timeout -k 10 120 python -u bench.py --op search --verify --no-cpu-baseline --steps 100 > $O/bench_$m.jsonl 2>> $O/bench.err
  tail -1 $O/bench_$m.jsonl
  LNX_PROF_SEARCH=$mm timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES -d $O/pmc_$m -o pmc --output-format csv -- python3 bench.py --op search --no-cpu-baseline --steps 3 --warmup 1 --prewarm-s 0 > $O/pmc_$m.log 2>&1
done
echo done
