# Round 4: batch polish schedules under one Ruiz pass (polish_from 25/50/75/100) on config 3
# (B=4096), config 4 (B=2048 = the 8-GPU shard, B=16384) and config 2; plus an output dump of the
# current build for bitwise A/B checks.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O/sched
timeout -k 10 200 python -u tools/dump_outputs.py $O/outputs_base.npz > $O/dump_base.log 2>&1 || exit 1
for pf in 75 25 50 100 75; do
  for c in "config3" "config4 --batch 2048" "config4" "config2"; do
    tag=$(echo "$c" | tr -d ' -')_pf$pf
    timeout -k 10 120 python bench.py --config $c --polish-from $pf --steps 20 --warmup 3 --cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --check-sample 64 > $O/sched/$tag.json 2> $O/sched/$tag.err || exit 1
  done
done
echo done
