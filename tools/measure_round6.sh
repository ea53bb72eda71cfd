# Round-6 measurement set, part A (TAG=r06_final): GPU tests, smoke, three runs of the driver's bench
# command, steady state, rocprofv3 kernel-trace stats (whole line and headline only), PMC passes on the
# headline launch.  Part B: tools/measure_round6b.sh.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_final}; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined --no-strong"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2>> $O/bench.err || exit 1; done &&
timeout -k 10 300 python bench.py $HEAD > $O/bench_steady.json 2>> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_head -o run -f csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 $HEAD > $O/bench_prof_head.json 2> $O/bench_prof_head.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc_req -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_req.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_sq -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/pmc_f64 -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_f64.log 2>&1
rc=$?; echo "exit $rc"; tail -2 $O/pytest_gpu.log; exit $rc
