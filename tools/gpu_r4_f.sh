#!/bin/bash
# Round 4: np8_assign_wide per-phase cycles (experiment build) in the C5 frozen and conjugate sweeps.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4f}
mkdir -p $OUT
for pu in frozen niw_conjugate; do
  NP8_LIB_OVERRIDE=noparama_amd/lib/exp/wph.so timeout -k 10 200 python -u bench.py --config C5 --param-update $pu --steps 20 --warmup 10 --cpu-seconds 0 > $OUT/$pu.json 2> $OUT/$pu.err || exit 1
  echo $pu; grep "assign_wide phases" $OUT/$pu.err | tail -3
done
echo F_DONE
