# PMC passes on the headline launch with the current library (keys profiles/pmc_traffic.json to its
# sha), then the default bench line (which then carries traffic / hw_flops), the small-batch sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc2; mkdir -p $O
HEAD="--cpu-seconds 0 --no-config1 --no-config5 --no-osqp-settings --no-pipelined"
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/pmc_req -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_req.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_sq -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/pmc_f64 -o run -f csv -- python3 $R/bench.py --steps 3 --warmup 1 $HEAD > $O/pmc_f64.log 2>&1 &&
cd $R && timeout -k 10 300 bash tools/diag/gpu_c2_batches.sh > $O/c2b.log 2>&1
rc=$?; echo "exit $rc"; exit $rc
