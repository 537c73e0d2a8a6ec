set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/prof/profile.sh r5n mtu1500 &&
bash tools/prof/profile.sh r5n zipf64_1500 &&
bash tools/prof/profile.sh r5n mtu1500 rx_verify &&
bash tools/prof/profile.sh r5n jumbo9000
