# A/B of a k_solve change: parity tests, lone-wave stamps (N=10), config 3 / config 2 against the previous
# library (tools/diag/libmpcqp_base.so), interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_params.py -x -v --timeout 200 --timeout-method thread > $O/ab_pytest.log 2>&1
rc=$?; tail -3 $O/ab_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/stamps.py config3 --horizon 10 --batch 1 > $O/ab_stamps_n10_one.json &&
timeout -k 10 120 python tools/stamps.py config3 --horizon 10 --batch 256 > $O/ab_stamps_n10_lone.json || exit 1
for r in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export MPCQP_LIB=$R/tools/diag/libmpcqp_base.so MPCQP_ABI_ANY=1; else unset MPCQP_LIB MPCQP_ABI_ANY; fi
    timeout -k 10 200 python bench.py --cpu-seconds 0 --no-config1 --no-config5 --check-sample 64 > $O/ab_${L}_c3_$r.json 2> $O/ab_${L}_c3_$r.err || exit 1
    timeout -k 10 200 python bench.py --config config2 --cpu-seconds 0 --no-config1 --check-sample 64 > $O/ab_${L}_c2_$r.json 2> $O/ab_${L}_c2_$r.err || exit 1
  done
done
unset MPCQP_LIB MPCQP_ABI_ANY
for f in $O/ab_*_c*_*.json; do python -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], round(d['value']), round(d['kernel_ms']['k_solve'],4), d.get('config1',{}).get('gpu_device_loop_ms_per_step'), d['rel_err'].get('iters_agreement'))"; done
python -c "import json;a=json.load(open('$O/ab_stamps_n10_one.json'));print({k:v for k,v in a.items() if k.startswith(('setup','qp'))})"
