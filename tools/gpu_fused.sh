set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/fz3_pytest.log 2>&1
rc=$?; tail -3 $O/fz3_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/fz3_bench.json 2> $O/fz3_bench.err &&
MPCQP_LIB=$R/tools/diag/libmpcqp_base.so MPCQP_ABI_ANY=1 timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz3_base_c3.json 2> $O/fz3_base_c3.err &&
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz3_new_c3.json 2> $O/fz3_new_c3.err
rc=$?
for f in $O/fz3_bench.json $O/fz3_*_c3.json; do python -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], round(d['value']), d['kernel_ms'])"; done
python -c "import json;d=json.load(open('$O/fz3_bench.json'));print(json.dumps(d['config1']))"
exit $rc
