set -o pipefail
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python tools/phase_timing.py > gpurun_out/phase.json 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run -f csv -- python3 $R/bench.py --steps 10 --warmup 2 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err
