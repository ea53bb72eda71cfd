# Config 2 / config 4 bench lines and the fleet closed-loop bench with the current kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 200 python bench.py --config config2 --cpu-seconds 5 > $O/bench_config2.json 2> $O/bench_config2.err &&
timeout -k 10 300 python bench.py --config config4 --cpu-seconds 5 > $O/bench_config4.json 2> $O/bench_config4.err &&
timeout -k 10 300 python -u tools/fleet_bench.py > $O/fleet_bench.json 2> $O/fleet_bench.err
echo "exit $?"
