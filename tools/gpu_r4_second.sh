# Round 4: the wide tests (the rest passed in the first call), smoke, bench, N=32, B=1 latency,
# N=20 stamps, qp_cycles.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu2.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 200 python bench.py --horizon 32 --steps 5 --warmup 2 --cpu-seconds 0 --no-config1 --no-osqp-settings --check-sample 128 > $O/bench_N32.json 2> $O/bench_N32.err &&
timeout -k 10 200 python -u tools/b1_latency.py > $O/b1_latency.json 2> $O/b1_latency.err &&
MPCQP_LIB=$R/diag_libs/libmpcqp_stamps20.so timeout -k 10 120 python -u tools/stamps.py config3 > $O/stamps_n20.json 2> $O/stamps.err &&
MPCQP_LIB=$R/diag_libs/libmpcqp_stamps20.so timeout -k 10 120 python -u tools/stamps.py config3 --worst 0 --by 1 > $O/stamps_n20_worst.json 2>> $O/stamps.err &&
timeout -k 10 200 python -u tools/qp_cycles.py > $O/qp_cycles.json 2> $O/qp_cycles.err
rc=$?; echo "exit $rc"; tail -3 $O/pytest_gpu2.log; exit $rc
