# Lone-wave phase stamps (one QP per CU) at N = 10 under the B=1 latency schedule and the batch default.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
MPCQP_LIB=$R/diag_libs/libmpcqp_stamps10.so timeout -k 10 120 python -u tools/stamps.py config3 --horizon 10 --batch 256 --polish-from 25 > $O/stamps10_lone_pf25.json 2> $O/stamps10.err &&
MPCQP_LIB=$R/diag_libs/libmpcqp_stamps10.so timeout -k 10 120 python -u tools/stamps.py config3 --horizon 10 --batch 256 > $O/stamps10_lone_pf75.json 2>> $O/stamps10.err
rc=$?; echo "exit $rc"; exit $rc
