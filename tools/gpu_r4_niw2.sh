#!/bin/bash
# Round 4: NIW posterior draws with one Philox call per normal quad -- NIW / wide GPU tests, the C5 conjugate line,
# and np8_niw_post's phase cycles (experiment build).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4niw2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_niw.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 10 --cpu-seconds 0"
timeout -k 10 300 python -u $B > $OUT/conj.json 2> $OUT/conj.err || exit 1
python -c "import json; d=json.loads(open('$OUT/conj.json').read().strip().splitlines()[-1]); print('conj', round(d['value']), 'sweeps/s', round(d['ms_per_step'], 3), 'ms')"
NP8_LIB_OVERRIDE=noparama_amd/lib/exp/niwt.so timeout -k 10 300 python -u $B > $OUT/niwt.out 2> $OUT/niwt.err || exit 1
grep "niw_post s=" $OUT/niwt.out | tail -3 || true
echo NIW2_DONE
