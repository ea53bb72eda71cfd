# Round-6 measurement set, part B (TAG=r06_final): the other configurations, long horizons, B=1 latency,
# iteration-counter agreement with the C restatement, gloo rehearsals of the N-rank line on one GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_final}; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --no-strong"
timeout -k 10 200 python bench.py --config config2 $HEAD > $O/c2.json 2> $O/c.err &&
timeout -k 10 200 python bench.py --config config4 --batch 2048 $HEAD > $O/c4_b2048.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --config config4 $HEAD > $O/c4_b16384.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 32 $HEAD --check-sample 128 > $O/N32.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 40 --steps 20 --warmup 20 $HEAD --check-sample 64 > $O/N40.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 48 --steps 20 --warmup 20 $HEAD --check-sample 32 > $O/N48.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 56 --steps 10 --warmup 5 $HEAD --check-sample 32 > $O/N56.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 64 --steps 10 --warmup 5 $HEAD --check-sample 32 > $O/N64.json 2>> $O/c.err &&
timeout -k 10 200 python -u tools/b1_latency.py > $O/b1_latency.json 2> $O/b1.err &&
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --cpu-seconds 3 > $O/gloo2.json 2> $O/gloo2.err &&
timeout -k 10 400 python bench.py --gpus 4 --backend gloo --steps 20 --warmup 5 --cpu-seconds 3 > $O/gloo4.json 2> $O/gloo4.err &&
timeout -k 10 600 python -u tools/iters_agreement.py > $O/iters_agreement.json 2> $O/iters.err
rc=$?; echo "exit $rc"; exit $rc
