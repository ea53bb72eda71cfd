set -o pipefail
PREFIX=n30 REPS=1 bash tools/diag/ab_cfg.sh > gpurun_out/ab_n30b.txt 2>&1 &&
for N in 32 40 48 63; do
timeout -k 10 200 python bench.py --config config3 --horizon $N --batch 4096 --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 --check-sample 32 > gpurun_out/wide_$N.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/wide_$N.json')); print($N, round(d['value']), round(d['kernel_ms']['k_solve'],3), d['solved_fraction'], d['rel_err']['max_rel_err_U'], d['iters_mean'])" >> gpurun_out/ab_n30b.txt
done
