#!/bin/bash
# Round 4: the NIW draw with its own factor (no np8_wide_rows in the conjugate sweep) and the two-wave
# np8_suffstats_wide -- the wide / NIW GPU tests, the C5 conjugate bench line, a kernel trace, the phase stamps.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4e}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_niw.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 10 --cpu-seconds 0"
timeout -k 10 300 python -u $B > $OUT/conj.json 2> $OUT/conj.err || exit 1
python -c "import json; d=json.loads(open('$OUT/conj.json').read().strip().splitlines()[-1]); print('conj', round(d['value']), 'sweeps/s', round(d['ms_per_step'], 3), 'ms', 'quad_forms/item', d['roofline']['executed']['quad_forms_per_item'])"
timeout -k 10 300 python -u bench.py --config C5 --steps 40 --warmup 10 --cpu-seconds 0 > $OUT/frozen.json 2> $OUT/frozen.err || exit 1
python -c "import json; d=json.loads(open('$OUT/frozen.json').read().strip().splitlines()[-1]); print('frozen', round(d['value']), 'sweeps/s', round(d['ms_per_step'], 3), 'ms assign', round(d['roofline']['assign_ms_per_launch'], 4), 'quad_forms/item', d['roofline']['executed']['quad_forms_per_item'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 $B > $OUT/tr.log 2>&1 || exit 1
python tools/trace_tail.py $OUT/tr 0.5 > $OUT/tr.txt || exit 1
head -12 $OUT/tr.txt
NP8_LIB_OVERRIDE=noparama_amd/lib/exp/niwt.so timeout -k 10 200 python -u $B > $OUT/niwt.json 2> $OUT/niwt.err || exit 1
grep "niw_post s=" $OUT/niwt.err | tail -4 || true
grep "wide_rows s=" $OUT/niwt.err | tail -6 || true
echo E_DONE
