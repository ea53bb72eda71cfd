# Round 4: fleet / swarm GPU tests after the reset changes, then the fleet benchmark (end to end and
# loop-only), paired and unpaired.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fleet.py tests/test_gpu_swarm.py tests/test_gpu_pair.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/fl_pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 16384 --horizon 15 --pairing off --reps 2 > $O/fl_fleet_off.json 2> $O/fl_fleet.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 16384 --horizon 15 --pairing auto --reps 2 > $O/fl_fleet_auto.json 2>> $O/fl_fleet.err
rc=$?; echo "exit $rc"; tail -2 $O/fl_pytest.log; exit $rc
