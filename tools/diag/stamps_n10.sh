# per-phase stamps of k_solve<10> (libmpcqp_stamps.so built with -DMPCQP_ONLY_N=10): lone waves and a full batch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py config3 --horizon 10 --batch 256 > gpurun_out/stamps_n10_lone.json &&
timeout -k 10 120 python tools/stamps.py config3 --horizon 10 --batch 1 > gpurun_out/stamps_n10_one.json &&
timeout -k 10 120 python tools/stamps.py config3 --horizon 10 > gpurun_out/stamps_n10_all.json
