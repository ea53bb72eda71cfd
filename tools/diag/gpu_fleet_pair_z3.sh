# The fused fleet loop at N = 15 with pairing off / auto on the final library (after the n <= 32
# broadcast change, which speeds the one-vehicle-per-wave kernel and leaves the paired one as it was).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fz3; mkdir -p $O
for rep in 1 2; do for m in off auto; do
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 16384 --pairing $m > $O/fleet_${m}_$rep.json 2>> $O/fleet.err || exit 1
done; done; echo done
