set -o pipefail
cd $GRAFT_REPO_ROOT
PYTHONPATH=. timeout -k 10 120 python -u tools/prof/tx_finish_parts.py > gpurun_out/r5q_parts.json 2>&1 &&
bash tools/prof/profile.sh r5q mtu1500 tx_finish
