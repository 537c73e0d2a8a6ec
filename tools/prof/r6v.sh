set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/prof/profile.sh r6v mtu1500 &&
bash tools/prof/profile.sh r6v zipf64_1500 &&
bash tools/prof/profile.sh r6v mtu1500 rx_verify &&
bash tools/prof/profile.sh r6v mtu1500 tx_finish &&
bash tools/prof/profile.sh r6v jumbo9000
