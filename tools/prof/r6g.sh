set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 120 python3 -c "
from lneto_amd import synth
import numpy as np
synth.zipf_lengths(1 << 20).astype(np.uint32).tofile('gpurun_out/zipf_len.u32')
" &&
timeout -k 10 200 ./tools/ubench/host_rows > gpurun_out/r6g_rows_256.jsonl 2>&1 &&
timeout -k 10 200 ./tools/ubench/host_rows gpurun_out/zipf_len.u32 > gpurun_out/r6g_rows_zipf.jsonl 2>&1
