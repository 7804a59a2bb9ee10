#!/bin/bash
# Round 4 profiles at HEAD: C3 (prof.sh), C5 (prof_c5.sh), the mixed regime (prof_mixed.sh), then the timed-region
# overhead of the driver's command (C3, --steps 20 / 100 / 400).
set -o pipefail
export TMPDIR=/tmp
bash tools/prof.sh gpurun_out/prof_r04 || exit 1
bash tools/prof_c5.sh gpurun_out/prof_r04_c5 || exit 1
bash tools/prof_mixed.sh gpurun_out/prof_r04_mixed || exit 1
OUT=gpurun_out/r4steps
mkdir -p $OUT
for k in 20 100 400; do
  timeout -k 10 200 python -u bench.py --steps $k --warmup 5 --cpu-seconds 0 --cold-sweeps 0 --no-c5 > $OUT/s$k.json 2> $OUT/s$k.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/s$k.json').read().strip().splitlines()[-1]); print('steps $k', round(d['value']), 'sweeps/s', round(d['ms_per_step'] * 1e3, 2), 'us/sweep')"
done
echo PROFALL_DONE
