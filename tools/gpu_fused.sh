# fused closed loop (k_fleet_loop): fleet / params / host GPU tests, k_solve<20> A/B against the
# previous library (tools/diag/libmpcqp_base.so), fleet bench stepped vs fused, config-1 loop fused
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fleet.py tests/test_gpu_params.py -x -v --timeout 200 --timeout-method thread > $O/fz_pytest.log 2>&1
rc=$?; tail -3 $O/fz_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz_new_c3.json 2> $O/fz_new_c3.err &&
MPCQP_LIB=$R/tools/diag/libmpcqp_base.so MPCQP_ABI_ANY=1 timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz_base_c3.json 2> $O/fz_base_c3.err &&
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz_new2_c3.json 2> $O/fz_new2_c3.err &&
timeout -k 10 300 python -u tools/fleet_bench.py > $O/fz_fleet_stepped.json 2> $O/fz_fleet_stepped.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused > $O/fz_fleet_fused.json 2> $O/fz_fleet_fused.err
rc=$?
for f in $O/fz_*_c3.json; do python -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], round(d['value']), d['kernel_ms'])"; done
tail -1 $O/fz_fleet_stepped.json; tail -1 $O/fz_fleet_fused.json
exit $rc
