set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
MPCQP_LIB=$R/tools/diag/libmpcqp_base.so MPCQP_ABI_ANY=1 timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz_base_c3.json 2> $O/fz_base_c3.err &&
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz_new2_c3.json 2> $O/fz_new2_c3.err &&
MPCQP_LIB=$R/tools/diag/libmpcqp_base.so MPCQP_ABI_ANY=1 timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --check-sample 64 > $O/fz_base2_c3.json 2> $O/fz_base2_c3.err &&
timeout -k 10 300 python -u tools/fleet_bench.py > $O/fz_fleet_stepped.json 2> $O/fz_fleet_stepped.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused > $O/fz_fleet_fused.json 2> $O/fz_fleet_fused.err
rc=$?
for f in $O/fz_*_c3.json; do python -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], round(d['value']), d['kernel_ms'])"; done
tail -1 $O/fz_fleet_stepped.json; tail -1 $O/fz_fleet_fused.json
exit $rc
