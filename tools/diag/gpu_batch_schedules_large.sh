# Polish schedule on large batches (many QPs per wave slot: the tail amortises, the mean cost counts)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for run in "config4 16384" "config3 65536" "config3 16384"; do
  set -- $run
  for pf in 150 100 75; do
    timeout -k 10 200 python bench.py --config $1 --batch $2 --set polish_from=$pf --steps 5 --warmup 2 --cpu-seconds 0 --no-config1 --no-config5 --check-sample 64 > $O/bl_$1_$2_$pf.json 2> $O/bl_$1_$2_$pf.err || exit 1
    python -c "import json;d=json.load(open('$O/bl_$1_$2_$pf.json'));print('$1', $2, $pf, round(d['value']), round(d['kernel_ms']['k_solve'],4))"
  done
done
