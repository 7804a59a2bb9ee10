#!/bin/bash
# Round 4: host-side split of the driver command's timed region (C3, --steps 20), three runs.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4o}
mkdir -p $OUT
for i in 1 2 3; do
  NP8_BENCH_PHASES=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --cold-sweeps 0 --no-c5 > $OUT/s$i.json 2> $OUT/s$i.err || exit 1
  grep "timed region" $OUT/s$i.err || true
done
NP8_BENCH_PHASES=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5 > $OUT/w40.json 2> $OUT/w40.err || exit 1
grep "timed region" $OUT/w40.err || true
echo O_DONE
