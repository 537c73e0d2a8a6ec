set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6q/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6q/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r6q/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6q/smoke.log 2>&1 && tail -1 gpurun_out/r6q/smoke.log &&
timeout -k 10 300 python -u bench.py > gpurun_out/r6q/bench_default.jsonl 2>&1 && tail -1 gpurun_out/r6q/bench_default.jsonl | cut -c1-300
