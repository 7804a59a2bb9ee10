#!/bin/bash
# Round 4: every wave's cycles of one np8_assign_wide launch (C5 frozen), fp32 screen against the bf16 screen.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4l}
mkdir -p $OUT
B="bench.py --config C5 --steps 4 --warmup 2 --cpu-seconds 0 --cold-sweeps 0"
for v in oldph curph; do
  NP8_LIB_OVERRIDE=noparama_amd/lib/exp/$v.so timeout -k 10 200 python -u $B > $OUT/$v.out 2> $OUT/$v.err || exit 1
  grep "^wq " $OUT/$v.out > $OUT/$v.wq || true
  wc -l $OUT/$v.wq
done
rm -f $OUT/*.out
echo L_DONE
