#!/bin/bash
# Development: time the tools/diag/libmpcqp_${PREFIX}*.so variants on one config (CONFIG, B).
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-2}; CONFIG=${CONFIG:-config4}; B=${B:-16384}; PREFIX=${PREFIX:-}
for r in $(seq $REPS); do
for lib in tools/diag/libmpcqp_${PREFIX}*.so; do
  v=$(basename $lib .so); v=${v#libmpcqp_}
  [ "$v" = stamps ] && continue
  MPCQP_ABI_ANY=1 MPCQP_LIB=$lib timeout -k 10 120 python bench.py --config $CONFIG --batch $B --steps 10 --warmup 2 --cpu-seconds 0 --no-config1 --check-sample 64 > gpurun_out/ab_${v}.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_${v}.json')); print('$v', $B, round(d['value']), round(d['kernel_ms']['k_solve'],4), d['solved_fraction'], d['rel_err']['max_rel_err_U'], d['rel_err']['active_set_mismatches'])"
done
done
