#!/bin/bash
# Round 4: C5 frozen A/B -- the committed build (lib/exp/head.so) against the working tree, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4g}
mkdir -p $OUT
B="bench.py --config C5 --steps 40 --warmup 10 --cpu-seconds 0"
for i in 1 2; do
  NP8_LIB_OVERRIDE=noparama_amd/lib/exp/head.so timeout -k 10 200 python -u $B > $OUT/head_$i.json 2> $OUT/head_$i.err || exit 1
  timeout -k 10 200 python -u $B > $OUT/cur_$i.json 2> $OUT/cur_$i.err || exit 1
done
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), "sweeps/s", round(d["ms_per_step"], 4), "ms, assign", round(d["roofline"]["assign_ms_per_launch"], 4))
PY
echo G_DONE
