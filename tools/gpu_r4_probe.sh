#!/bin/bash
# Round-4 probe (one GPU call): per-wave phase stamps of np8_assign_fast at the C4 shard sizes, and a kernel
# trace of the 125k-item sweep (per-kernel averages and the gaps between dispatches of a graph replay).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4probe}
mkdir -p $OUT
for n in 125000 1000000; do
  NP8_LIB_OVERRIDE=noparama_amd/lib/exp/clk.so timeout -k 10 180 python -u tools/clocks.py $n warm > $OUT/clk_$n.json 2> $OUT/clk_$n.err || exit 1
done
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5 --n 125000"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr125k -o run -- python3 bench.py $A > $OUT/tr125k.log 2>&1 || exit 1
python tools/trace_tail.py $OUT/tr125k 0.5 $OUT/tr125k_tail.json > $OUT/tr125k_tail.txt || exit 1
echo PROBE_DONE
