# A/B of a fused-loop (k_fleet_loop) change against tools/diag/libmpcqp_base.so: fleet / params
# parity tests, then config-1 device loop and the fused fleet bench, interleaved new / base.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fleet.py tests/test_gpu_params.py tests/test_gpu_swarm.py -x -v --timeout 200 --timeout-method thread > $O/abl_pytest.log 2>&1
rc=$?; tail -3 $O/abl_pytest.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export MPCQP_LIB=$R/tools/diag/libmpcqp_base.so MPCQP_ABI_ANY=1; else unset MPCQP_LIB MPCQP_ABI_ANY; fi
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-config5 --check-sample 64 > $O/abl_${L}_$r.json 2> $O/abl_${L}_$r.err || exit 1
    timeout -k 10 200 python -u tools/fleet_bench.py --fused --vehicles 1 100 1024 > $O/abl_${L}_fleet_$r.json 2> $O/abl_${L}_fleet_$r.err || exit 1
  done
done
unset MPCQP_LIB MPCQP_ABI_ANY
for f in $O/abl_new_1.json $O/abl_base_1.json $O/abl_new_2.json $O/abl_base_2.json; do python -c "import json;d=json.load(open('$f'));c=d['config1'];print('$f'.split('/')[-1], round(d['kernel_ms']['k_solve'],4), round(c['gpu_device_loop_ms_per_step'],5), c['device_loop_max_state_diff_px'])"; done
for f in $O/abl_*_fleet_*.json; do python -c "
import json
l=[x for x in open('$f') if x.strip()][-1]; d=json.loads(l)
print('$f'.split('/')[-1], [(r['vehicles'], round(r['seconds']*1e3,3)) for r in d['runs']])"; done
