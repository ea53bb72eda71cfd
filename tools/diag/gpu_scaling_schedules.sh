# Ruiz passes (scaling) x polish schedule on the batch configs, measured
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for cfg in config3 config2 config4; do
  for sp in "10 150" "1 150" "1 100" "1 75"; do
    set -- $sp
    timeout -k 10 200 python bench.py --config $cfg --set scaling=$1 --set polish_from=$2 --steps 10 --warmup 2 --cpu-seconds 0 --no-config1 --no-config5 --check-sample 128 > $O/ss_${cfg}_$1_$2.json 2> $O/ss_${cfg}_$1_$2.err || exit 1
    python -c "import json;d=json.load(open('$O/ss_${cfg}_$1_$2.json'));r=d['rel_err'];print('$cfg', 'scaling', $1, 'polish_from', $2, round(d['value']), round(d['kernel_ms']['k_solve'],4), r['iters_agreement'], r['max_rel_err_U'], r['active_set_mismatches'], r['status_mismatches'])"
  done
done
