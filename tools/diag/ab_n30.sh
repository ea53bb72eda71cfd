#!/bin/bash
# Development: config4 (N=30, B=16384) timing of the N=30 kernel variants.
set -o pipefail
mkdir -p gpurun_out
for v in n30old n30new; do
  MPCQP_ABI_ANY=1 MPCQP_LIB=tools/diag/libmpcqp_$v.so timeout -k 10 200 python bench.py --config config4 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/ab4_$v.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab4_$v.json')); print('$v', round(d['value']), round(d['kernel_ms']['k_solve'],4), d['iters_mean'], d['solved_fraction'])"
done
