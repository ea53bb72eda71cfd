# GPU test suite + smoke + default bench line.   gpurun --timeout 600 -- 'bash tools/gpu_tests.sh'
# Exits non-zero when the tests, the smoke or the bench fail.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
brc=$?
echo "pytest $rc bench $brc"
exit $(( rc != 0 ? rc : brc ))
