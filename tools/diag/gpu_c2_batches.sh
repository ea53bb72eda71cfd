# Config 2 (identical QPs) at 256 / 512 / 1024 / 2048 per GPU: lone-wave latency vs SIMD sharing.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 16"
for B in 256 512 1024 2048 4096; do
timeout -k 10 120 python bench.py --config config2 --batch $B $HEAD >> $O/c2b.json 2>> $O/c2b.err || exit 1
done; echo done
