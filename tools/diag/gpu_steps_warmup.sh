# bench.py's headline at several step / warmup counts (clock ramp, steady state)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
SIDE="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 64"
for sw in "20 3" "20 20" "100 20" "200 50" "20 3" "100 100"; do set -- $sw
timeout -k 10 120 python bench.py --steps $1 --warmup $2 $SIDE >> $O/sw.json 2>> $O/sw.err || exit 1
done; echo done
