# Round 4: pairing in the throughput regime (fleet of 16384 vehicles) and the rocprofv3 kernel trace
# of the paired batch kernel (N = 15, B = 16384) beside the unpaired one.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
SIDE="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 64"
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 4096 16384 --horizon 15 --pairing off --reps 2 > $O/pair2_fleet_off.json 2> $O/pair2_fleet.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 4096 16384 --horizon 15 --pairing on --reps 2 > $O/pair2_fleet_on.json 2>> $O/pair2_fleet.err
rc=$?; echo "exit $rc"; exit $rc
