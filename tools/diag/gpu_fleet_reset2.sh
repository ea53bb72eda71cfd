# Fleet reset after the shared path packing (start states read from the packed plans): the fleet /
# swarm / refbuild GPU tests, the reset breakdown, and the fused fleet bench end to end at N = 15.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fr2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fleet.py tests/test_gpu_swarm.py tests/test_gpu_refbuild.py tests/test_gpu_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -u tools/diag/fleet_reset_timing.py > $O/reset_timing.json 2> $O/reset.err &&
for rep in 1 2; do
timeout -k 10 300 python -u tools/fleet_bench.py --fused --vehicles 1024 4096 16384 > $O/fleet_auto_$rep.json 2>> $O/fleet.err || exit 1
done; echo done
