#!/bin/bash
# Round 4: np8_assign_wide per-phase cycles, committed build against the working tree (C5 frozen).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4h}
mkdir -p $OUT
B="bench.py --config C5 --steps 20 --warmup 10 --cpu-seconds 0"
for v in headph wph; do
  NP8_LIB_OVERRIDE=noparama_amd/lib/exp/$v.so timeout -k 10 200 python -u $B > $OUT/$v.json 2> $OUT/$v.err || exit 1
  echo $v; grep "assign_wide phases" $OUT/$v.json | tail -2 || true
done
echo H_DONE
