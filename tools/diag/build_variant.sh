#!/bin/bash
# Development: single-horizon (N=20) build of the library for A/B timing of kernel variants.
#   bash tools/diag/build_variant.sh NAME [extra hipcc flags]  -> tools/diag/libmpcqp_NAME.so
#   MPCQP_LIB=tools/diag/libmpcqp_NAME.so python bench.py --cpu-seconds 0
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -DMPCQP_ONLY_N=${ONLY_N:-20} "$@" \
  -o tools/diag/libmpcqp_$name.so rrt-mpc_amd/csrc/mpcqp.hip rrt-mpc_amd/csrc/mpcqp_fleet.hip rrt-mpc_amd/csrc/mpcqp_refbuild.hip rrt-mpc_amd/csrc/mpcqp_rrt.hip rrt-mpc_amd/csrc/mpcqp_inflate.hip rrt-mpc_amd/csrc/mpcqp_wide.hip rrt-mpc_amd/csrc/mpcqp_swarm.hip
