#!/bin/bash
# Round 4: kernel traces of the C5 frozen sweep, committed build (lib/exp/head.so) against the working tree.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4i}
mkdir -p $OUT
B="bench.py --config C5 --steps 20 --warmup 10 --cpu-seconds 0"
NP8_LIB_OVERRIDE=noparama_amd/lib/exp/oldscreen.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/old -o run -- python3 $B > $OUT/old.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cur -o run -- python3 $B > $OUT/cur.log 2>&1 || exit 1
for v in old cur; do echo $v; python tools/trace_tail.py $OUT/$v 0.5 > $OUT/$v.txt && head -6 $OUT/$v.txt; done
echo I_DONE
