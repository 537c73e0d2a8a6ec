# ingress verdicts: workgroups per CU sweep
set -e
O=gpurun_out/ingress_grid
mkdir -p $O
# LNX_PROF_* knobs are read by the research library only
export LNETO_AMD_LIB=$PWD/lneto_amd/liblneto_amd_research.so
for g in 64 96 128 256 100000; do
  LNX_PROF_INGRESS_WG_PER_CU=$g timeout -k 10 120 python -u bench.py --op ingress --no-cpu-baseline --steps 100 > $O/bench_$g.jsonl 2>> $O/bench.err
done
echo done
