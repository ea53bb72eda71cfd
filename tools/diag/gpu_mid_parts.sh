# Mid kernel: 2 column parts (product default at NT <= 48) vs 4 (diag_libs/libmpcqp_mid_p4.so) at
# N = 33 / 40 / 44 / 48, config-3 generator, B = 4096; every run spot-checked against the C restatement.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 64 --steps 20 --warmup 10"
for N in 40 33 48 44; do
timeout -k 10 200 python bench.py --horizon $N $HEAD >> $O/midp_base.json 2>> $O/midp.err || exit 1
MPCQP_LIB=$R/diag_libs/libmpcqp_mid_p4.so timeout -k 10 200 python bench.py --horizon $N $HEAD >> $O/midp_p4.json 2>> $O/midp.err || exit 1
done; echo done
