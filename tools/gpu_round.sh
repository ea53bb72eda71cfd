# One GPU call: parity tests, smoke, bench, kernel-trace profile, PMC passes (HBM bytes, SQ, FP64),
# config 4 at the 8-GPU shard (B=2048), B=4096 and B=16384.
# usage: gpurun --timeout 1100 -- 'bash tools/gpu_round.sh'
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 $R/bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-config5 > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-config5 > $O/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc_req -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-config5 > $O/pmc_req.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_sq -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-config5 > $O/pmc_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/pmc_f64 -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-config5 > $O/pmc_f64.log 2>&1 &&
cd $R &&
timeout -k 10 200 python bench.py --config config4 --batch 2048 --cpu-seconds 0 --no-config1 > $O/c4_b2048.json 2> $O/c4.err &&
timeout -k 10 200 python bench.py --config config4 --batch 4096 --cpu-seconds 0 --no-config1 > $O/c4_b4096.json 2>> $O/c4.err &&
timeout -k 10 200 python bench.py --config config4 --cpu-seconds 0 --no-config1 > $O/c4_b16384.json 2>> $O/c4.err
rc=$?; echo "exit $rc"; exit $rc
