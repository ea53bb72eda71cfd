set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/list_avail.txt 2>&1 || true
grep -i -E "SQC|IFETCH|ICACHE|INST_LEVEL|WAIT_INST|SQ_INSTS_BRANCH" $O/list_avail.txt | head -80 > $O/list_icache.txt || true
echo done
