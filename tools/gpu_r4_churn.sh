#!/bin/bash
# Round 4: churn mode (parallel lists + in-graph re-sort while many items move) -- GPU tests touching graphs, cold
# start and the mixed regime, then the default bench's warm / cold / mixed legs.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4churn}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_fold.py tests/test_gpu_parity.py tests/test_gpu_resume.py tests/test_gpu_fast_split.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
A="--steps 20 --warmup 5 --cpu-seconds 0 --no-c5"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1]); c=d['cold_start']; print('warm', round(d['value']), 'cold', round(c['value']), 'mixed_ms', round(c['mixed']['ms_per_sweep'], 4))"
done
echo CHURN_DONE
