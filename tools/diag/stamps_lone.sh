# per-phase stamps: full batch and lone waves (256 QPs, one per CU).  gpurun -- 'bash tools/diag/stamps_lone.sh'
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py config3 > gpurun_out/stamps_all.json &&
timeout -k 10 120 python tools/stamps.py config3 --batch 256 > gpurun_out/stamps_lone.json
