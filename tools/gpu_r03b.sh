# round 3: mid-horizon kernel smoke + tests + benches; swarm parity; config-4 shard lines
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 120 python -u tools/diag/mid_smoke.py 32 40 > $O/r03b_mid_smoke.log 2>&1 &&
timeout -k 10 120 python -u tools/diag/mid_smoke.py 48 56 63 >> $O/r03b_mid_smoke.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -v --timeout 200 --timeout-method thread > $O/r03b_pytest_wide.log 2>&1 ;
rc1=$?
timeout -k 10 200 python bench.py --horizon 40 --cpu-seconds 0 --no-config1 --check-sample 64 > $O/r03b_bench_N40.json 2> $O/r03b_bench_N40.err ;
timeout -k 10 200 python bench.py --horizon 32 --cpu-seconds 0 --no-config1 --check-sample 64 > $O/r03b_bench_N32.json 2> $O/r03b_bench_N32.err ;
timeout -k 10 200 python bench.py --horizon 63 --cpu-seconds 0 --no-config1 --check-sample 64 > $O/r03b_bench_N63.json 2> $O/r03b_bench_N63.err ;
echo "wide tests rc $rc1"; tail -3 $O/r03b_pytest_wide.log; cat $O/r03b_mid_smoke.log
