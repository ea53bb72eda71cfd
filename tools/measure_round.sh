# The measurement set of a round on the current library: GPU tests, smoke, the driver's bench command, rocprofv3
# kernel trace (whole line and headline only), PMC passes on the headline launch, config lines.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-round}; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --no-strong"
# the sweep microbenchmark when it was built here beforehand (hipcc --offload-arch=gfx950 -O3 -o
# tools/micro/sweep_bench tools/micro/sweep_bench.hip)
{ [ ! -x tools/micro/sweep_bench ] || timeout -k 10 120 tools/micro/sweep_bench > $O/sweep_bench.json 2> $O/sweep_bench.err; } &&
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py $HEAD > $O/bench_steady.json 2>> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run -f csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 $HEAD > $O/bench_prof_head.json 2> $O/bench_prof_head.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc_req -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_req.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_sq -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/pmc_f64 -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_f64.log 2>&1 &&
cd $R &&
timeout -k 10 200 python bench.py --config config2 $HEAD > $O/c2.json 2> $O/c.err &&
timeout -k 10 200 python bench.py --config config4 --batch 2048 $HEAD > $O/c4_b2048.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --config config4 $HEAD > $O/c4_b16384.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 32 $HEAD --check-sample 128 > $O/N32.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 40 --steps 20 --warmup 10 $HEAD --check-sample 64 > $O/N40.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 48 --steps 10 --warmup 5 $HEAD --check-sample 32 > $O/N48.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 56 --steps 10 --warmup 5 $HEAD --check-sample 32 > $O/N56.json 2>> $O/c.err &&
timeout -k 10 200 python bench.py --horizon 64 --steps 10 --warmup 5 $HEAD --check-sample 32 > $O/N64.json 2>> $O/c.err &&
timeout -k 10 200 python -u tools/b1_latency.py > $O/b1_latency.json 2> $O/b1.err &&
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 > $O/gloo2.json 2> $O/gloo2.err
rc=$?; echo "exit $rc"; tail -2 $O/pytest_gpu.log; exit $rc
