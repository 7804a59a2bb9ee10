#!/bin/bash
# C5 niw_conjugate: wide / NIW GPU tests, the bench line and a kernel trace (round-4 blocked factor kernels).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4c5b}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_niw.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 10 --cpu-seconds 0"
timeout -k 10 300 python -u $B > $OUT/conj.json 2> $OUT/conj.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o run -- python3 $B > $OUT/tr.log 2>&1 || exit 1
python tools/trace_tail.py $OUT/tr 0.5 > $OUT/tr.txt || exit 1
head -10 $OUT/tr.txt
python -c "import json; d=json.loads(open('$OUT/conj.json').read().strip().splitlines()[-1]); print('conj', round(d['value']), 'sweeps/s', round(d['ms_per_step'], 3), 'ms')"
echo C5B_DONE
