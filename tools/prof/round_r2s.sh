# r2s: 2-rank rehearsal of the N>1 bench path (both ranks share the box's one GPU; configs[4] slices)
set -e
O=gpurun_out/r2s
mkdir -p $O
LNETO_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload mtu1500_x8 --steps 20 --warmup 3 > $O/bench_n2_shared_gpu.jsonl 2> $O/bench_n2.err
echo done
