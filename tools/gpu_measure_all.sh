# Every measured workload with the current kernels (one GPU call):
#   gpurun --timeout 1100 -- 'bash tools/gpu_measure_all.sh'
# config 2 / config 4 bench lines, long horizons (mid / wide kernels), the reproducible mode, the
# fleet closed loop (stepped and fused), the iteration agreement with the C restatement and the
# config-5 swarm bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 200 python bench.py --config config2 --cpu-seconds 5 > $O/bench_config2.json 2> $O/bench_config2.err &&
timeout -k 10 300 python bench.py --config config4 --cpu-seconds 5 > $O/bench_config4.json 2> $O/bench_config4.err &&
timeout -k 10 200 python bench.py --set reproducible=1 --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 > $O/bench_reproducible.json 2> $O/bench_reproducible.err &&
for N in 32 40 63; do
  timeout -k 10 200 python bench.py --horizon $N --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 --check-sample 64 > $O/bench_N$N.json 2> $O/bench_N$N.err || exit 1
done &&
timeout -k 10 300 python -u tools/fleet_bench.py > $O/fleet_bench.json 2> $O/fleet_bench.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused > $O/fleet_bench_fused.json 2> $O/fleet_bench_fused.err &&
timeout -k 10 500 python -u tools/iters_agreement.py > $O/iters_agreement.json 2> $O/iters_agreement.err &&
timeout -k 10 300 python -u tools/swarm_bench.py > $O/swarm_bench.json 2> $O/swarm_bench.err &&
timeout -k 10 300 python -u tools/swarm_bench.py --fused > $O/swarm_bench_fused.json 2> $O/swarm_bench_fused.err
echo "exit $?"
