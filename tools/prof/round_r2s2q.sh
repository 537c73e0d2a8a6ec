# r2s2q: segment-mode CRC against offsets mode by slot layout (tools/prof/seg_probe.py)
set -e
O=gpurun_out/r2s2q
mkdir -p $O
timeout -k 10 300 python -u tools/prof/seg_probe.py > $O/seg_probe.txt 2>&1
echo done
