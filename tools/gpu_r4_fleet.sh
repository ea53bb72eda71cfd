# Round 4: fleet / swarm GPU tests after the reset changes, then the fleet benchmark (end to end and
# loop-only), paired and unpaired.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
true &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 16384 --horizon 15 --pairing off --reps 5 > $O/fl_fleet_off.json 2> $O/fl_fleet.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 16384 --horizon 15 --pairing auto --reps 5 > $O/fl_fleet_auto.json 2>> $O/fl_fleet.err
rc=$?; echo "exit $rc"; tail -2 $O/fl_pytest.log; exit $rc
