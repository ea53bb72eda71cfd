# Round 4: the whole GPU suite, smoke and the default bench line on the current library.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/g_pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/g_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/g_bench.json 2> $O/g_bench.err
rc=$?; echo "exit $rc"; tail -3 $O/g_pytest_gpu.log; exit $rc
