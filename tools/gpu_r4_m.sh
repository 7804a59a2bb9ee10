#!/bin/bash
# Round 4: the wide / NIW GPU tests, then the C5 frozen and niw_conjugate bench lines and a kernel trace of the
# conjugate sweep (NIW draw with its own factor, Sigma^8 eigenvalue bound, fp32 exact-distance screen).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4m}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_niw.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for pu in frozen niw_conjugate; do
  timeout -k 10 300 python -u bench.py --config C5 --param-update $pu --steps 20 --warmup 10 --cpu-seconds 0 > $OUT/$pu.json 2> $OUT/$pu.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/$pu.json').read().strip().splitlines()[-1]); print('$pu', round(d['value']), 'sweeps/s', round(d['ms_per_step'], 3), 'ms assign', round(d['roofline']['assign_ms_per_launch'], 4), 'quad_forms/item', d['roofline']['executed']['quad_forms_per_item'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 10 --cpu-seconds 0 > $OUT/tr.log 2>&1 || exit 1
python tools/trace_tail.py $OUT/tr 0.5 > $OUT/tr.txt || exit 1
head -8 $OUT/tr.txt
echo M_DONE
