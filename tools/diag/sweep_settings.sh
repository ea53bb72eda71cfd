#!/bin/bash
# Development: k_solve time vs solver settings (config3 N=20 B=4096).  Args: KEY VALUE...
set -o pipefail
mkdir -p gpurun_out
key=$1; shift
for v in "$@"; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --set $key=$v > gpurun_out/ss_$v.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ss_$v.json')); print('$key', '$v', round(d['value']), round(d['kernel_ms']['k_solve'],4), d['iters_mean'])"
done
