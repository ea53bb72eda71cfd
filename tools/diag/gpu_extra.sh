set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
timeout -k 10 300 python tools/fleet_bench.py > $O/fleet_bench.json 2> $O/fleet_bench.err &&
timeout -k 10 300 python tools/swarm_bench.py > $O/swarm_bench.json 2> $O/swarm_bench.err &&
timeout -k 10 200 python bench.py --config config4 --cpu-seconds 0 > $O/bench_config4.json 2> $O/bench_config4.err &&
timeout -k 10 200 python bench.py --config config2 --cpu-seconds 0 > $O/bench_config2.json 2> $O/bench_config2.err
echo "exit $?"
