set -o pipefail
PREFIX=n30 bash tools/diag/ab_cfg.sh > gpurun_out/ab_n30.txt 2>&1 &&
PREFIX=n20 CONFIG=config3 B=4096 REPS=3 bash tools/diag/ab_cfg.sh > gpurun_out/ab_n20.txt 2>&1
