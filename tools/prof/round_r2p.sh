# r2p: jumbo frames: product against its loads-only (1) and math-only (2) forms; the 1500-B product too
set -e
O=gpurun_out/r2p
mkdir -p $O
timeout -k 10 300 python -u tools/prof/variants.py jumbo9000 0,1,2,15,16 7 > $O/var_jumbo.log 2>&1
timeout -k 10 300 python -u tools/prof/timeline.py jumbo9000 0 > $O/timeline_jumbo.txt 2>&1
echo done
