# Multi-rank rehearsal of bench.py's distributed path on one GPU (gloo; the driver's 8-GPU run uses
# RCCL): 4 ranks weak scaling, 2 ranks strong scaling (config 4).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 4 --backend gloo --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_gloo4_weak.json 2> $O/bench_gloo4_weak.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29552 bench.py --gpus 2 --backend gloo --config config4 --global-batch 16384 --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_gloo2_strong.json 2> $O/bench_gloo2_strong.err
echo "exit $?"
