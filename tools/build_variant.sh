#!/bin/bash
# A/B experiments: build libnp8.so with extra preprocessor flags into noparama_amd/lib/exp/<name>.so
# usage: tools/build_variant.sh <name> <flags...>; load with NP8_LIB_OVERRIDE=<path>
set -e
name=$1; shift
cd "$(dirname "$0")/../noparama_amd/csrc"
out=../lib/exp/$name
mkdir -p $out
F="--offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -Wall $*"
for f in np8_kernels np8_niw np8_wide np8_sm np8_capi; do
  /opt/rocm/bin/hipcc $F -c $f.hip -o $out/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../lib/exp/$name.so $out/*.o -lrccl
rm -rf $out
echo built ../lib/exp/$name.so
