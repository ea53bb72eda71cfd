# Pbar packed (N >= 24, 2 waves per SIMD up to N = 31) against the previous library: parity tests at
# N = 24..31, then config 4 (N = 30) and config 3 at N = 24 / 28 / 30 with both libraries.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; T=${TAG:-pk}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_params.py -x -v --timeout 200 --timeout-method thread > $O/${T}_pytest.log 2>&1
rc=$?; tail -3 $O/${T}_pytest.log
[ $rc -ne 0 ] && exit $rc
for L in new base; do
  if [ $L = base ]; then export MPCQP_LIB=$R/tools/diag/libmpcqp_base.so; fi
  timeout -k 10 200 python bench.py --config config4 --cpu-seconds 0 --no-config1 --check-sample 64 > $O/${T}_${L}_c4.json 2> $O/${T}_${L}_c4.err || exit $?
  for N in 24 28 30; do
    timeout -k 10 200 python bench.py --horizon $N --cpu-seconds 0 --no-config1 --check-sample 64 > $O/${T}_${L}_N$N.json 2> $O/${T}_${L}_N$N.err || exit $?
  done
done
unset MPCQP_LIB
for f in $O/${T}_*_c4.json $O/${T}_*_N*.json; do python -c "import json,sys;d=json.load(open('$f'));print('$f'.split('/')[-1], round(d['value']), d['kernel_ms'], d['rel_err'].get('max_rel_err_U'), d['rel_err'].get('iters_agreement'))"; done
