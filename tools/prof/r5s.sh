set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
V=$PWD/tools/prof/_var/lib768.so
timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r5s_parts_1024.json 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r5s_parts_768.json 2>&1 &&
timeout -k 10 180 python -u bench.py --op rx_verify --steps 50 --no-cpu-baseline > gpurun_out/r5s_rxv_1024.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 180 python -u bench.py --op rx_verify --steps 50 --no-cpu-baseline > gpurun_out/r5s_rxv_768.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 180 python -u bench.py --op tx_finish --steps 50 --no-cpu-baseline > gpurun_out/r5s_txf_768.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 180 python -u bench.py --op rx_verify --workload zipf64_1500 --steps 20 --no-cpu-baseline > gpurun_out/r5s_rxv_zipf_768.jsonl 2>&1 &&
timeout -k 10 180 python -u bench.py --op rx_verify --workload zipf64_1500 --steps 20 --no-cpu-baseline > gpurun_out/r5s_rxv_zipf_1024.jsonl 2>&1
