#!/bin/bash
# Round 4: the full GPU suite and the C4 sizes (gpu_r4_check.sh), the driver command's timed-region split
# (gpu_r4_o.sh), and the C5 frozen / niw_conjugate lines.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r4_check.sh || exit 1
bash tools/gpu_r4_o.sh || exit 1
OUT=gpurun_out/r4p
mkdir -p $OUT
for pu in frozen niw_conjugate; do
  timeout -k 10 300 python -u bench.py --config C5 --param-update $pu --steps 20 --warmup 10 --cpu-seconds 0 > $OUT/$pu.json 2> $OUT/$pu.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/$pu.json').read().strip().splitlines()[-1]); print('$pu', round(d['value']), 'sweeps/s', round(d['ms_per_step'], 3), 'ms assign', round(d['roofline']['assign_ms_per_launch'], 4), 'quad_forms/item', d['roofline']['executed']['quad_forms_per_item'])"
done
echo P_DONE
