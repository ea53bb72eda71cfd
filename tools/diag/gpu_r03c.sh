set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 120 python -u tools/diag/mid_x.py 32 > $O/r03c_mid_x.log 2>&1 ;
timeout -k 10 200 python -u tools/diag/mid_stamps.py run 32 40 63 > $O/r03c_mid_stamps.json 2> $O/r03c_mid_stamps.err ;
cat $O/r03c_mid_x.log; cat $O/r03c_mid_stamps.json | head -60
