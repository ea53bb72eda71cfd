# k_solve<20> rate against batch size (config 3's QP distribution): where the dispatch tail stops mattering
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for B in 2048 4096 8192 16384 65536 262144; do
  timeout -k 10 200 python bench.py --batch $B --steps 5 --warmup 2 --cpu-seconds 0 --no-config1 --no-config5 --check-sample 64 > $O/sweep_B$B.json 2> $O/sweep_B$B.err || exit 1
  python -c "import json;d=json.load(open('$O/sweep_B$B.json'));print($B, round(d['value']), round(d['kernel_ms']['k_solve'],4), d['roofline']['frac'])"
done
