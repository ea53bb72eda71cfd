set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/stamps.py config3 > gpurun_out/stamps_all.json &&
timeout -k 10 120 python tools/stamps.py config3 --worst 0 --batch 256 > gpurun_out/stamps_worst0.json &&
timeout -k 10 120 python tools/stamps.py config3 --worst 0 --by 1 --batch 256 > gpurun_out/stamps_polish0.json &&
timeout -k 10 120 python tools/stamps.py config3 --worst 10 --by 1 --batch 256 > gpurun_out/stamps_polish10.json
