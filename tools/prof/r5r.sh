set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r5r_parts_1024.json 2>&1 &&
LNETO_AMD_LIB=$PWD/tools/prof/_var/lib768.so timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r5r_parts_768.json 2>&1 &&
LNETO_AMD_LIB=$PWD/tools/prof/_var/lib512.so timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r5r_parts_512.json 2>&1 &&
timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r5r_parts_1024b.json 2>&1
