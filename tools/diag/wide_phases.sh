set -o pipefail
for S in "" "--set polish=0" "--set polish_from=0 --set polish_near=0.0" "--set max_iter=1 --set polish=0" "--set max_iter=25 --set polish=0" "--method newton"; do
timeout -k 10 200 python bench.py --config config3 --horizon 32 --batch 4096 --steps 2 --warmup 1 --cpu-seconds 0 --no-config1 --check-sample 0 $S > gpurun_out/wp.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/wp.json')); print('$S', round(d['kernel_ms']['k_solve'],3), d['iters_mean'], d['solved_fraction'])" >> gpurun_out/wide_phases.txt
done
