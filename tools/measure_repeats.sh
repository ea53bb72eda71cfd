# repeats of the driver command and the near-target configs on one box (run-to-run spread)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-repeats}; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --no-strong"
for i in 1 2 3; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2>> $O/err.txt || exit 1
timeout -k 10 200 python bench.py --config config2 $HEAD > $O/c2_$i.json 2>> $O/err.txt || exit 1
timeout -k 10 200 python bench.py --config config4 --batch 2048 $HEAD > $O/c4_b2048_$i.json 2>> $O/err.txt || exit 1
timeout -k 10 200 python -u tools/b1_latency.py > $O/b1_latency_$i.json 2>> $O/err.txt || exit 1
done
echo done
