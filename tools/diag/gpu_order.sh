# fused-loop dispatch order: fleet / swarm tests, fleet and swarm benches (fused)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fleet.py tests/test_gpu_swarm.py -x -v --timeout 300 --timeout-method thread > $O/or_pytest.log 2>&1
rc=$?; tail -3 $O/or_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 100 1024 4096 8192 16384 > $O/or_fleet_fused.json 2> $O/or_fleet_fused.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --vehicles 8192 16384 > $O/or_fleet_stepped_big.json 2> $O/or_fleet_stepped_big.err &&
timeout -k 10 300 python -u tools/swarm_bench.py --fused > $O/or_swarm_fused.json 2> $O/or_swarm_fused.err
rc=$?
head -5 $O/or_fleet_fused.json | cut -c1-200; head -2 $O/or_fleet_stepped_big.json | cut -c1-200; head -2 $O/or_swarm_fused.json | cut -c1-200
exit $rc
