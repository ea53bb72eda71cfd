# reproducible mode: its GPU tests and its bench line (config3 B=4096 N=20)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_fleet.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_wide.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-config1 --set reproducible=1 > $O/bench_repro.json 2> $O/bench_repro.err
echo "exit $?"
