#!/bin/bash
# A/B variant of np8_kernels.hip (run here, on the CPU): builds noparama_amd/lib_exp/<name>/libnp8.so from
# np8_kernels.hip compiled with extra flags (only the D = 8, M = 3 instances with -DNP8_EXP_ONLY_D8), linked with the
# other objects of the in-tree build (make first).  Select it on the GPU box with NP8_LIB_OVERRIDE=<path>.
#   tools/ab_build.sh <name> [hipcc flags ...]
set -euo pipefail
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/noparama_amd/csrc
LIB=$ROOT/noparama_amd/lib
OUT=$ROOT/noparama_amd/lib_exp/$name
mkdir -p "$OUT"
FLAGS="--offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -Wall"
/opt/rocm/bin/hipcc $FLAGS "$@" -c "$SRC/np8_kernels.hip" -o "$OUT/np8_kernels.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libnp8.so" "$OUT/np8_kernels.o" "$LIB/np8_niw.o" \
    "$LIB/np8_wide.o" "$LIB/np8_sm.o" "$LIB/np8_rt.o" "$LIB/np8_capi.o" -lrccl
echo "$OUT/libnp8.so"
