set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5m_gpu_suite.log 2>&1 || { echo SUITE_FAILED; tail -40 gpurun_out/r5m_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r5m_gpu_suite.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5m_smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/r5m_smoke.log; exit 1; }
cat gpurun_out/r5m_smoke.log | tail -1
