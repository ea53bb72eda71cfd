# mid-horizon kernel: smoke, the long-horizon tests, benches at N = 32 / 40 / 48 / 63
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; T=${TAG:-mid}
timeout -k 10 120 python -u tools/diag/mid_smoke.py 32 40 48 63 > $O/${T}_smoke.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -v --timeout 200 --timeout-method thread > $O/${T}_pytest_wide.log 2>&1 ;
rc1=$?
case $rc1 in 124|134|137|139) echo "wide tests died rc $rc1"; tail -30 $O/${T}_pytest_wide.log; exit $rc1;; esac
for N in 32 40 48 63; do
  timeout -k 10 200 python bench.py --horizon $N --cpu-seconds 0 --no-config1 --check-sample 64 > $O/${T}_bench_N$N.json 2> $O/${T}_bench_N$N.err || break
done
echo "wide tests rc $rc1"; tail -3 $O/${T}_pytest_wide.log; cat $O/${T}_smoke.log
for N in 32 40 48 63; do python -c "import json;d=json.load(open('$O/${T}_bench_N$N.json'));print($N, round(d['value']), d['kernel_ms'], d['rel_err']['max_rel_err_U'], d['rel_err']['iters_agreement'])"; done
