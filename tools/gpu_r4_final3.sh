# Round 4 closing measurement set (3rd: after the n <= 32 broadcast change) on the final library: all GPU tests, smoke, the default bench line,
# its rocprofv3 kernel trace (and a headline-only one, whose k_solve<20> average is the headline's
# alone), PMC passes on the headline launch, config 2 / 4 lines, horizons 32 / 40 / 64 / 128, two QPs
# per wave at N = 15 / 10, the B=1 breakdown.
# usage: gpurun --timeout 1150 -- 'bash tools/gpu_r4_final3.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/final3; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 $R/bench.py --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run -f csv -- python3 $R/bench.py $HEAD > $O/bench_prof_head.json 2> $O/bench_prof_head.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc_req -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_req.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_sq -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/pmc_f64 -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_f64.log 2>&1 &&
cd $R &&
timeout -k 10 200 python bench.py --config config2 --cpu-seconds 0 --no-config1 > $O/c2.json 2> $O/c2.err &&
timeout -k 10 200 python bench.py --config config4 --batch 2048 --cpu-seconds 0 --no-config1 > $O/c4_b2048.json 2> $O/c4.err &&
timeout -k 10 200 python bench.py --config config4 --batch 4096 --cpu-seconds 0 --no-config1 > $O/c4_b4096.json 2>> $O/c4.err &&
timeout -k 10 200 python bench.py --config config4 --cpu-seconds 0 --no-config1 > $O/c4_b16384.json 2>> $O/c4.err &&
timeout -k 10 200 python bench.py --horizon 32 --cpu-seconds 0 --no-config1 --no-osqp-settings --check-sample 128 > $O/N32.json 2> $O/N.err &&
timeout -k 10 200 python bench.py --horizon 40 --steps 20 --warmup 10 --cpu-seconds 0 --no-config1 --no-osqp-settings --check-sample 128 > $O/N40.json 2>> $O/N.err &&
timeout -k 10 200 python bench.py --horizon 64 --steps 3 --warmup 1 --cpu-seconds 0 --no-config1 --no-osqp-settings --no-pipelined --check-sample 32 > $O/N64.json 2>> $O/N.err &&
timeout -k 10 300 python bench.py --horizon 128 --batch 1024 --steps 2 --warmup 1 --cpu-seconds 0 --no-config1 --no-osqp-settings --no-pipelined --check-sample 8 > $O/N128.json 2>> $O/N.err &&
for N in 15 10; do for m in off on; do
timeout -k 10 120 python bench.py --horizon $N --batch 16384 --pairing $m $HEAD --check-sample 128 > $O/pair_N${N}_$m.json 2>> $O/pair.err || exit 1
done; done &&
timeout -k 10 200 python -u tools/b1_latency.py > $O/b1_latency.json 2> $O/b1_latency.err &&
timeout -k 10 300 python -u tools/fleet_bench.py --fused --horizon 10 --vehicles 1 100 1024 > $O/fleet_n10.json 2> $O/fleet.err
rc=$?; echo "exit $rc"; tail -2 $O/pytest_gpu.log; exit $rc
