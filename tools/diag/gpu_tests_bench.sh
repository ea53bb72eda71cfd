set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "maxsize|FAIL|Error" $O/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['kernel_ms'], {k:v for k,v in d['config1'].items() if 'ms' in k})"
exit $rc
