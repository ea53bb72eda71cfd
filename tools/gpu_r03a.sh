# round 3: swarm parity (host-only checkers), bench with iteration agreement, config-4 shard shapes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_swarm.py tests/test_gpu_pipeline.py -v --timeout 200 --timeout-method thread > $O/r03a_pytest.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/r03a_bench.json 2> $O/r03a_bench.err &&
timeout -k 10 200 python bench.py --config config4 --batch 2048 --cpu-seconds 0 --no-config1 > $O/r03a_c4_b2048.json 2> $O/r03a_c4.err &&
timeout -k 10 200 python bench.py --config config4 --batch 4096 --cpu-seconds 0 --no-config1 > $O/r03a_c4_b4096.json 2>> $O/r03a_c4.err &&
timeout -k 10 200 python bench.py --config config4 --cpu-seconds 0 --no-config1 > $O/r03a_c4_b16384.json 2>> $O/r03a_c4.err
rc=$?; tail -3 $O/r03a_pytest.log; echo "exit $rc"; exit $rc
