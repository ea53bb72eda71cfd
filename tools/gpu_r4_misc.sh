# Round 4: B=1 schedules (config 1), pipelined batches, N = 64 / 128 lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 200 python -u tools/b1_schedules.py > $O/b1_schedules.json 2> $O/b1_schedules.err &&
timeout -k 10 200 python -u tools/pipelined.py > $O/pipelined.json 2> $O/pipelined.err &&
timeout -k 10 200 python bench.py --horizon 64 --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 --no-osqp-settings --check-sample 32 > $O/bench_N64.json 2> $O/bench_N64.err &&
timeout -k 10 300 python bench.py --horizon 128 --batch 1024 --steps 2 --warmup 1 --cpu-seconds 0 --no-config1 --no-osqp-settings --check-sample 8 > $O/bench_N128.json 2> $O/bench_N128.err
rc=$?; echo "exit $rc"; exit $rc
