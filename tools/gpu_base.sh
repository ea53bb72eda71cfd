set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err
echo "exit $?"
