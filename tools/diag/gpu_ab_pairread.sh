# A/B of the pair kernel's cross-lane reads by v_readlane (Lanes<true>::readv) instead of ds_bpermute:
# the candidate library (diag_libs/libmpcqp_cand.so) against the product one -- outputs bit for bit
# (paired workloads included), the GPU suite on the candidate, then paired batches and the paired
# fused fleet, each as base, new, base, new.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abp; mkdir -p $O
NEW=$R/diag_libs/libmpcqp_cand.so
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --check-sample 64"
timeout -k 10 200 python -u tools/dump_outputs.py $O/out_base.npz > $O/dump.log 2>&1 &&
MPCQP_LIB=$NEW timeout -k 10 200 python -u tools/dump_outputs.py $O/out_new.npz >> $O/dump.log 2>&1 &&
python tools/dump_outputs.py --compare $O/out_base.npz $O/out_new.npz > $O/compare.txt 2>&1
cat $O/compare.txt
MPCQP_LIB=$NEW timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_new.txt 2>&1 || { tail -20 $O/pytest_new.txt; exit 1; }
tail -1 $O/pytest_new.txt
for rep in 1 2; do for lib in base new; do
  if [ $lib = new ]; then export MPCQP_LIB=$NEW; else unset MPCQP_LIB; fi
  timeout -k 10 120 python bench.py --horizon 15 --batch 16384 $HEAD >> $O/p15_$lib.json 2>> $O/ab.err &&
  timeout -k 10 120 python bench.py --horizon 10 --batch 16384 $HEAD >> $O/p10_$lib.json 2>> $O/ab.err &&
  timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 4096 16384 --reps 3 >> $O/fleet_$lib.json 2>> $O/ab.err || exit 1
done; done
unset MPCQP_LIB; echo done
