# Round 4, first GPU call: tests, smoke, bench line, B=1 latency breakdown, N=20 phase stamps,
# the N=32 line (now the one-wave kernel).
#   gpurun --timeout 1100 -- 'bash tools/gpu_r4_first.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python bench.py --horizon 32 --steps 5 --warmup 2 --cpu-seconds 0 --no-config1 --no-osqp-settings --check-sample 128 > $O/bench_N32.json 2> $O/bench_N32.err &&
timeout -k 10 200 python -u tools/b1_latency.py > $O/b1_latency.json 2> $O/b1_latency.err &&
MPCQP_LIB=$R/diag_libs/libmpcqp_stamps20.so timeout -k 10 120 python -u tools/stamps.py config3 > $O/stamps_n20.json 2> $O/stamps.err &&
MPCQP_LIB=$R/diag_libs/libmpcqp_stamps20.so timeout -k 10 120 python -u tools/stamps.py config3 --worst 0 --by 1 > $O/stamps_n20_worst.json 2>> $O/stamps.err
rc=$?; echo "exit $rc"; tail -3 $O/pytest_gpu.log; exit $rc
