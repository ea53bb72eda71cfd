set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread > $O/ag_pytest.log 2>&1
rc=$?; tail -3 $O/ag_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/iters_agreement.py > $O/iters_agreement.json 2> $O/iters_agreement.err
