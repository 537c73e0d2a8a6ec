# r2s2r: segment-mode lean rows with every step non-temporal (LNX_PROF_SEG_EP=0) against the edge policy (EP = 1)
set -e
O=gpurun_out/r2s2r
mkdir -p $O
timeout -k 10 300 python -u tools/prof/seg_probe.py > $O/seg_probe_ep1.txt 2>&1
LNX_PROF_SEG_EP=0 timeout -k 10 300 python -u tools/prof/seg_probe.py > $O/seg_probe_ep0.txt 2>&1
LNX_PROF_SEG_EP=0 timeout -k 10 300 python -u -m pytest tests/test_tx.py -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_ep0.log 2>&1
echo done
