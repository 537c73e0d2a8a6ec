set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
V=$PWD/tools/prof/_var/libgather.so
R="bench.py --op rx_ring --workload zipf64_1500 --steps 10 --warmup 2"
LNETO_AMD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_rx_ring.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r6i_tests.log 2>&1 || { tail -20 gpurun_out/r6i_tests.log; exit 1; }
tail -1 gpurun_out/r6i_tests.log
timeout -k 10 240 python -u $R > gpurun_out/r6i_inplace_1.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $R > gpurun_out/r6i_gather_1.jsonl 2>&1 &&
LNETO_AMD_LIB=$V timeout -k 10 240 python -u $R > gpurun_out/r6i_gather_2.jsonl 2>&1 &&
timeout -k 10 240 python -u $R > gpurun_out/r6i_inplace_2.jsonl 2>&1 &&
timeout -k 10 200 python3 -c "
from lneto_amd import synth
import numpy as np
synth.zipf_lengths(1 << 20).astype(np.uint32).tofile('gpurun_out/zipf_len.u32')
" &&
timeout -k 10 200 ./tools/ubench/host_rows gpurun_out/zipf_len.u32 > gpurun_out/r6i_rows_zipf.jsonl 2>&1
