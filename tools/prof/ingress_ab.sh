# A/B: the ingress verdict / TX generate rows (product) against the form
# LNX_PROF_INGRESS_UNROLL=U selects (default 24: the r1g dword lanes; r3n ran
# it against a per-wave buffer-descriptor build, see
# profiles/r3n_ingress_buffer_loads_rejected.txt), after the parity tests;
# three alternating bench runs of each.
#   tools/prof/ingress_ab.sh TAG [U]
set -e
O=gpurun_out/ingress_ab_$1
mkdir -p $O
# LNX_PROF_* knobs are read by the research library only
export LNETO_AMD_LIB=$PWD/lneto_amd/liblneto_amd_research.so
timeout -k 10 300 python -u -m pytest tests/test_ingress.py tests/test_rx_ring.py tests/test_tx_checksum.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
for op in ingress tx_checksum; do
  for i in 1 2 3; do
    LNX_PROF_INGRESS_UNROLL=${2:-24} timeout -k 10 120 python -u bench.py --op $op --no-cpu-baseline --steps 100 > $O/${op}_alt_$i.jsonl 2>> $O/bench.err
    timeout -k 10 120 python -u bench.py --op $op --no-cpu-baseline --steps 100 > $O/${op}_product_$i.jsonl 2>> $O/bench.err
  done
done
python3 - $O <<'PY'
import glob, json, sys
o = sys.argv[1]
for f in sorted(glob.glob(o + "/*.jsonl")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
