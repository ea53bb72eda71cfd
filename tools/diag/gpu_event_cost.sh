set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
SIDE="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 64 --steps 100 --warmup 5"
for c in "config3" "config2"; do for e in 1 1000 1 1000; do
timeout -k 10 120 python bench.py --config $c --event-every $e $SIDE >> $O/ev_$c.json 2>> $O/ev.err || exit 1
done; done; echo done
