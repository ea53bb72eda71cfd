# Small batches (<= one wave per SIMD): config 2 (identical QPs) at 256 / 512 / 1024 / 2048, and
# config 2 / 3 / 4 at B = 1024 under the batch polish schedule (75) and the latency one (25).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 16"
for B in 256 512 1024 2048; do
timeout -k 10 120 python bench.py --config config2 --batch $B $HEAD >> $O/c2b.json 2>> $O/c2b.err || exit 1
done
for c in config2 config3 config4; do for pf in 75 25; do
timeout -k 10 120 python bench.py --config $c --batch 1024 --polish-from $pf $HEAD >> $O/c2b_pf.json 2>> $O/c2b.err || exit 1
done; done; echo done
