set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -v --timeout 200 --timeout-method thread > $O/pytest_wide.log 2>&1; rc=$?
tail -25 $O/pytest_wide.log | grep -E "PASS|FAIL|Error|passed|failed"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for N in 32 40 48 63; do
  timeout -k 10 200 python bench.py --horizon $N --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 --check-sample 64 > $O/bench_N$N.json 2> $O/bench_N$N.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_N$N.json')); print($N, round(d['value']), round(d['kernel_ms']['k_solve'],3), d['solved_fraction'], d['rel_err']['max_rel_err_U'], d['rel_err']['active_set_mismatches'], d['iters_mean'])"
done
