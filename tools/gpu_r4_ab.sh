#!/bin/bash
# A/B of the round-4 launch reductions at the C4 shard sizes, plus a kernel trace of the default build at 125k items.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4ab}
mkdir -p $OUT
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
for n in ${SIZES:-125000 1000000}; do
  for v in def off; do
    if [ $v = off ]; then E="NP8_NO_LLFOLD=1 NP8_LISTS_ALWAYS=1 NP8_SORT_IN_GRAPH=1"; else E=""; fi
    env $E timeout -k 10 200 python -u bench.py $A --n $n > $OUT/${v}_$n.json 2> $OUT/${v}_$n.err || exit 1
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 bench.py $A --n 125000 > $OUT/tr.log 2>&1 || exit 1
python tools/trace_tail.py $OUT/tr 0.5 $OUT/tr_tail.json > $OUT/tr_tail.txt || exit 1
cat $OUT/tr_tail.txt
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/*_*.json")):
    if "tail" in f: continue
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), "sweeps/s", round(d["ms_per_step"] * 1e3, 2), "us/sweep, assign_us",
          round(d["roofline"]["assign_ms_per_launch"] * 1e3, 2))
PY
echo AB_DONE
