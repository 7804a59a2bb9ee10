#!/bin/bash
# Round 4: a variant library (lib/exp/sym.so: symmetric squarings in np8_niw_post) -- NIW / wide GPU tests through it,
# then the C5 conjugate line against the tree's library, alternating.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4sym}
mkdir -p $OUT
NP8_LIB_OVERRIDE=noparama_amd/lib/exp/sym.so timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_niw.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 10 --cpu-seconds 0"
for i in 1 2; do
  for v in base sym; do
    if [ $v = sym ]; then L=noparama_amd/lib/exp/sym.so; else L=noparama_amd/lib/libnp8.so; fi
    NP8_LIB_OVERRIDE=$L timeout -k 10 300 python -u $B > $OUT/$v$i.json 2> $OUT/$v$i.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'sweeps/s')"
  done
done
echo SYM_DONE
