# r1g GPU session h (lean-row product): 2-rank rehearsal of the N>1 bench path on one GPU, other ops' bench lines
set -e
mkdir -p gpurun_out/r1g
export LNETO_BENCH_SHARE_GPU=1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload mtu1500_x8 --steps 20 --warmup 3 > gpurun_out/r1g/bench_n2_shared_gpu.jsonl 2> gpurun_out/r1g/bench_n2.err
unset LNETO_BENCH_SHARE_GPU
timeout -k 10 200 python -u bench.py --op fcs_verify --no-cpu-baseline > gpurun_out/r1g/bench_fcs_verify_mtu1500.jsonl 2>> gpurun_out/r1g/ops.err
timeout -k 10 200 python -u bench.py --op sum16 --no-cpu-baseline > gpurun_out/r1g/bench_sum16_mtu1500.jsonl 2>> gpurun_out/r1g/ops.err
timeout -k 10 200 python -u bench.py --op ingress --no-cpu-baseline > gpurun_out/r1g/bench_ingress_mtu1500.jsonl 2>> gpurun_out/r1g/ops.err
timeout -k 10 200 python -u bench.py --with-copies --no-cpu-baseline > gpurun_out/r1g/bench_with_copies_mtu1500.jsonl 2>> gpurun_out/r1g/ops.err
timeout -k 10 200 python -u bench.py --op rx_ring > gpurun_out/r1g/bench_rx_ring.jsonl 2>> gpurun_out/r1g/ops.err
