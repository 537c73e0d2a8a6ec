set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
V=$PWD/tools/prof/_var/libh768.so
E="bench.py --op egress_packets --bufs slots --workload zipf64_1500 --steps 10 --warmup 2"
for i in 1 2 3; do
timeout -k 10 240 python -u $E > gpurun_out/r5y_e1024_$i.jsonl 2>&1 || exit 1
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $E > gpurun_out/r5y_e768_$i.jsonl 2>&1 || exit 1
done
