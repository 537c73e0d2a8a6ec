# GPU A/B run: parity tests, then the CRC kernel's variants per workload
# (usage: bash tools/prof/run_ab.sh "mtu1500:0,10,11 jumbo9000:0,10" [reps])
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
for spec in $1; do
  timeout -k 10 150 python -u tools/prof/variants.py ${spec%%:*} ${spec##*:} ${2:-7} >> gpurun_out/var.log 2>&1
done
