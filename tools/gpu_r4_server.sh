# Round 4: the B=1 server -- GPU tests from the pipeline file on, bench line, B=1 latency breakdown.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_planning.py tests/test_gpu_refbuild.py tests/test_gpu_swarm.py tests/test_gpu_wide.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu3.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke3.log 2>&1 &&
timeout -k 10 200 python -u tools/b1_latency.py > $O/b1_latency3.json 2> $O/b1_latency3.err &&
timeout -k 10 300 python bench.py > $O/bench3.json 2> $O/bench3.err
rc=$?; echo "exit $rc"; tail -3 $O/pytest_gpu3.log; exit $rc
