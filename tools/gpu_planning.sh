set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_planning.py tests/test_gpu_swarm.py -x -v --timeout 120 --timeout-method thread > $O/pytest_plan.log 2>&1 &&
timeout -k 10 300 python -u tools/swarm_bench.py > $O/swarm_bench.json 2> $O/swarm_bench.err
echo "exit $?"
