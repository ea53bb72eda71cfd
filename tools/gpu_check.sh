# One GPU call: the GPU test suite, smoke, the default bench line, a 2-rank gloo rehearsal of
# bench.py's distributed body on the one GPU, and the per-phase stamps breakdown.
# usage: gpurun --timeout 900 -- 'bash tools/gpu_check.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 > $O/bench_gloo2.json 2> $O/bench_gloo2.err &&
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --backend gloo --config config4 --global-batch 16384 --steps 3 --warmup 1 > $O/bench_gloo2_strong.json 2> $O/bench_gloo2_strong.err &&
timeout -k 10 120 python tools/stamps.py config3 > $O/stamps_all.json 2> $O/stamps.err
echo "exit $?"
