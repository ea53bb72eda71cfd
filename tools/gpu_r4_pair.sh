# Round 4: two QPs per wave (N <= 15) -- bitwise tests against the one-QP-per-wave kernel, the
# fleet / swarm suites (auto pairing past the wave slots), then paired vs unpaired throughput.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
SIDE="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 128"
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_fleet.py tests/test_gpu_swarm.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pair_pytest.log 2>&1 &&
for N in 15 10; do for B in 4096 16384; do for m in off on; do
timeout -k 10 120 python bench.py --horizon $N --batch $B --pairing $m $SIDE > $O/pair_N${N}_B${B}_$m.json 2>> $O/pair_bench.err || exit 1
done; done; done &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 --horizon 15 --pairing off > $O/pair_fleet_off.json 2> $O/pair_fleet.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 --horizon 15 --pairing on > $O/pair_fleet_on.json 2>> $O/pair_fleet.err
rc=$?; echo "exit $rc"; tail -3 $O/pair_pytest.log; exit $rc
