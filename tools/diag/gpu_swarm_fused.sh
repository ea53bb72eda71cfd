# fused swarm loop: swarm + fleet GPU tests, swarm bench stepped vs fused
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_swarm.py tests/test_gpu_fleet.py -x -v --timeout 300 --timeout-method thread > $O/sf_pytest.log 2>&1
rc=$?; tail -3 $O/sf_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/swarm_bench.py > $O/sf_swarm_stepped.json 2> $O/sf_swarm_stepped.err &&
timeout -k 10 300 python -u tools/swarm_bench.py --fused > $O/sf_swarm_fused.json 2> $O/sf_swarm_fused.err
rc=$?
head -2 $O/sf_swarm_stepped.json; head -2 $O/sf_swarm_fused.json
exit $rc
