#!/bin/bash
# A/B against an earlier commit: build libnp8.so from noparama_amd/csrc (and include/) as of <rev> into
# noparama_amd/lib/exp/<name>.so (load with NP8_LIB_OVERRIDE).  usage: tools/build_rev.sh <rev> <name> [flags]
set -e
rev=$1; name=$2; shift 2
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d)
git -C "$root" archive "$rev" noparama_amd/csrc include | tar -x -C "$tmp"
cd "$tmp/noparama_amd/csrc"
F="--offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -Wall $*"
for f in $(ls *.hip | sed "s/\.hip$//"); do /opt/rocm/bin/hipcc $F -c $f.hip -o $f.o & done
wait
mkdir -p "$root/noparama_amd/lib/exp"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$root/noparama_amd/lib/exp/$name.so" *.o -lrccl
rm -rf "$tmp"
echo "built noparama_amd/lib/exp/$name.so from $rev"
