# Two ranks on the one GPU over gloo (a rehearsal of the driver's multi-GPU bench path: weak scaling,
# then config 4 strong scaling).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --steps 20 --warmup 20 > $O/gloo2_weak.json 2> $O/gloo2.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --backend gloo --config config4 --global-batch 16384 --steps 20 --warmup 20 > $O/gloo2_strong.json 2>> $O/gloo2.err
rc=$?; echo "exit $rc"; exit $rc
