# Instruction-cache counters of the bench kernel (one --pmc pass).  gpurun -- 'bash tools/diag/pmc_icache.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAVES -d $O/pmc_icache -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 > $O/pmc_icache.log 2>&1
echo "exit $?"
