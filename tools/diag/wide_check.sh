set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_wide.py > gpurun_out/wide_tests.txt 2>&1 && \
timeout -k 10 120 python tools/diag/wide_stamps.py 32 512 > gpurun_out/wide_stamps.json 2>gpurun_out/wide_stamps.err && \
timeout -k 10 200 python bench.py --config config3 --horizon 32 --batch 4096 --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 --check-sample 0 > gpurun_out/wide_bench.json 2>gpurun_out/wide_bench.err
for N in 40 48 63; do
timeout -k 10 200 python bench.py --config config3 --horizon $N --batch 4096 --steps 2 --warmup 1 --cpu-seconds 0 --no-config1 --check-sample 0 > gpurun_out/wide_bench_$N.json 2>>gpurun_out/wide_bench.err || exit 1
done
