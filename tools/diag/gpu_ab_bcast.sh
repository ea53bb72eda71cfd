# A/B of the whole-wave broadcast at n <= 32 (rows 2-3 are padding: no permlane32 stage; no lane
# moves at n <= 16): the candidate library (diag_libs/libmpcqp_cand.so) against the product one --
# outputs bit for bit, the GPU suite on the candidate, then the N <= 16 latency / batch legs, each
# as base, new, base, new.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/abb; mkdir -p $O
NEW=$R/diag_libs/libmpcqp_cand.so
HEAD="--cpu-seconds 0 --no-config5 --no-osqp-settings --no-pipelined --check-sample 64"
timeout -k 10 200 python -u tools/dump_outputs.py $O/out_base.npz > $O/dump.log 2>&1 &&
MPCQP_LIB=$NEW timeout -k 10 200 python -u tools/dump_outputs.py $O/out_new.npz >> $O/dump.log 2>&1 &&
python tools/dump_outputs.py --compare $O/out_base.npz $O/out_new.npz > $O/compare.txt 2>&1
cat $O/compare.txt
MPCQP_LIB=$NEW timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_new.txt 2>&1 || { tail -20 $O/pytest_new.txt; exit 1; }
tail -1 $O/pytest_new.txt
for rep in 1 2; do for lib in base new; do
  if [ $lib = new ]; then export MPCQP_LIB=$NEW; else unset MPCQP_LIB; fi
  timeout -k 10 200 python -u tools/b1_latency.py >> $O/b1_$lib.json 2>> $O/ab.err &&
  timeout -k 10 200 python -u tools/b1_latency.py --horizon 15 >> $O/b1n15_$lib.json 2>> $O/ab.err &&
  timeout -k 10 120 python bench.py --horizon 10 --batch 1024 $HEAD >> $O/n10_$lib.json 2>> $O/ab.err &&
  timeout -k 10 120 python bench.py --horizon 15 --batch 1024 --no-config1 $HEAD >> $O/n15_$lib.json 2>> $O/ab.err &&
  timeout -k 10 200 python -u tools/fleet_bench.py --fused --horizon 10 --vehicles 1 100 1024 --reps 3 >> $O/fleet_$lib.json 2>> $O/ab.err || exit 1
done; done
unset MPCQP_LIB; echo done
