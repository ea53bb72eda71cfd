#!/bin/bash
# Development: time every tools/diag/libmpcqp_*.so variant (config3 N=20) at B=512 and 4096,
# interleaved over REPS rounds (clock drift shows up as spread, not as a variant difference).
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2}
for r in $(seq $REPS); do
for lib in tools/diag/libmpcqp_*.so; do
  v=$(basename $lib .so); v=${v#libmpcqp_}
  [ "$v" = stamps ] && continue
  for B in 512 4096; do
    MPCQP_ABI_ANY=1 MPCQP_LIB=$lib timeout -k 10 120 python bench.py --batch $B --steps 20 --warmup 3 --cpu-seconds 0 --no-config1 --check-sample 0 > gpurun_out/ab_${v}_$B.json || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_${v}_$B.json')); print('$v', $B, round(d['value']), round(d['kernel_ms']['k_solve'],4), d['solved_fraction'])"
  done
done
done
