# Polish schedule on the batch configs (config 2: one QP per wave slot; config 3: two): the tail-tuned
# default (polish_from 150) against earlier schedules, measured
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for cfg in config2 config3; do
  for pf in 150 100 75 50; do
    timeout -k 10 200 python bench.py --config $cfg --set polish_from=$pf --steps 10 --warmup 2 --cpu-seconds 0 --no-config1 --no-config5 --check-sample 64 > $O/bs_${cfg}_$pf.json 2> $O/bs_${cfg}_$pf.err || exit 1
    python -c "import json;d=json.load(open('$O/bs_${cfg}_$pf.json'));print('$cfg', $pf, round(d['value']), round(d['kernel_ms']['k_solve'],4))"
  done
done
