# Swarm (config 5) tests and bench.   gpurun --timeout 600 -- 'bash tools/gpu_swarm.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_swarm.py tests/test_gpu_planning.py tests/test_gpu_refbuild.py tests/test_gpu_fleet.py -v --timeout 300 --timeout-method thread > $O/pytest_swarm.log 2>&1
rc=$?
tail -5 $O/pytest_swarm.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u tools/swarm_bench.py > $O/swarm_bench.json 2> $O/swarm_bench.err
echo "exit $? pytest $rc"
