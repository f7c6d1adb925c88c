#!/bin/bash
# Build a library variant on the CPU host: tools/build_variant.sh NAME "EXTRA flags"
# -> franka-force-feedback-mpc_amd/lib/NAME/libffddp.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/franka-force-feedback-mpc_amd/lib/$1
make -s -B -C $R/franka-force-feedback-mpc_amd/csrc OUT=../lib/$1/libffddp.so EXTRA="$2"
