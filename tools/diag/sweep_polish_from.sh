#!/bin/bash
# Development: k_solve time vs the early-polish start iteration (config3 N=20 B=4096).
set -o pipefail
mkdir -p gpurun_out
for T in 0 75 100 125 150 200 300; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --polish-from $T > gpurun_out/pf_$T.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pf_$T.json')); print('polish_from', $T, round(d['value']), round(d['kernel_ms']['k_solve'],4), d['iters_mean'])"
done
