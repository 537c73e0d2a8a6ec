# sum16 workgroups-per-CU sweep (larger grids)
set -e
O=gpurun_out/grid_sweep2
mkdir -p $O
# LNX_PROF_* knobs are read by the research library only
export LNETO_AMD_LIB=$PWD/lneto_amd/liblneto_amd_research.so
for g in 256 512 1024 100000 256; do
  LNX_PROF_SUM16_WG_PER_CU=$g timeout -k 10 120 python -u bench.py --op sum16 --no-cpu-baseline --steps 100 > $O/bench_sum16_$g.jsonl 2>> $O/bench.err
done
echo done
