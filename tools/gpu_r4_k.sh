#!/bin/bash
# Round 4: np8_assign_wide timing variants (C5 frozen kernel trace): old fp32 screen, bf16 screen, and two probes.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4k}
mkdir -p $OUT
B="bench.py --config C5 --steps 10 --warmup 5 --cpu-seconds 0 --cold-sweeps 0"
for v in oldscreen vC vD cur; do
  if [ $v = cur ]; then L=noparama_amd/lib/libnp8.so; else L=noparama_amd/lib/exp/$v.so; fi
  NP8_LIB_OVERRIDE=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 $B > $OUT/$v.log 2>&1 || exit 1
  echo $v $(grep -h "assign_wide" $OUT/$v/run_kernel_stats.csv | cut -d, -f1-4)
done
echo K_DONE
