# Sharded config 5: the GPU test and a 2-rank gloo rehearsal of the distributed swarm bench on one GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_swarm.py -m gpu -x -v --timeout 240 --timeout-method thread -k sharded > $O/pytest_swarm_sharded.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 tools/swarm_bench.py --distributed --backend gloo --vehicles 100 1024 > $O/swarm_dist_gloo2.json 2> $O/swarm_dist_gloo2.err
echo "exit $?"
