# A/B of a kernel change that claims the same arithmetic: the candidate library
# (diag_libs/libmpcqp_setup_new.so) against the product one -- outputs bit for bit, then headline /
# config 2 / config 4 shard / B=1 latency, each as base, new, base, new.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab; mkdir -p $O
NEW=$R/diag_libs/libmpcqp_setup_new.so
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 64"
timeout -k 10 200 python -u tools/dump_outputs.py $O/out_base.npz > $O/dump.log 2>&1 &&
MPCQP_LIB=$NEW timeout -k 10 200 python -u tools/dump_outputs.py $O/out_new.npz >> $O/dump.log 2>&1 &&
python tools/dump_outputs.py --compare $O/out_base.npz $O/out_new.npz > $O/compare.txt 2>&1 &&
for rep in 1 2; do for lib in base new; do
  if [ $lib = new ]; then export MPCQP_LIB=$NEW; else unset MPCQP_LIB; fi
  timeout -k 10 120 python bench.py $HEAD >> $O/c3_$lib.json 2>> $O/ab.err &&
  timeout -k 10 120 python bench.py --config config2 $HEAD >> $O/c2_$lib.json 2>> $O/ab.err &&
  timeout -k 10 120 python bench.py --config config4 --batch 2048 $HEAD >> $O/c4_$lib.json 2>> $O/ab.err &&
  timeout -k 10 200 python -u tools/b1_latency.py >> $O/b1_$lib.json 2>> $O/ab.err || exit 1
done; done
unset MPCQP_LIB; echo done
