#!/bin/bash
# Development: k_solve time vs the near-tolerance early-polish ratio (config3 N=20 B=4096, config4).
set -o pipefail
mkdir -p gpurun_out
for R in 0 1.5 2 3 5 10; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --polish-near $R > gpurun_out/pn_$R.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pn_$R.json')); print('near', $R, round(d['value']), round(d['kernel_ms']['k_solve'],4), d['iters_mean'])"
done
for R in 0 3; do
  timeout -k 10 200 python bench.py --config config4 --steps 5 --warmup 1 --cpu-seconds 0 --polish-near $R > gpurun_out/pn4_$R.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pn4_$R.json')); print('config4 near', $R, round(d['value']), round(d['kernel_ms']['k_solve'],4), d['iters_mean'])"
done
