#!/bin/bash
# Round 4: the C5 conjugate sweep with the eigenvalue bound with one squaring more (experiment s4.so) against Sigma^8 (three).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4s4}
mkdir -p $OUT
B="bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 10 --cpu-seconds 0"
for i in 1 2; do
  for v in s8 s4; do
    if [ $v = s4 ]; then L=noparama_amd/lib/exp/s4.so; else L=noparama_amd/lib/libnp8.so; fi
    NP8_LIB_OVERRIDE=$L timeout -k 10 300 python -u $B > $OUT/$v$i.json 2> $OUT/$v$i.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'sweeps/s assign', round(d['roofline']['assign_ms_per_launch'], 4), 'quad', d['roofline']['executed']['quad_forms_per_item'])"
  done
done
echo S4_DONE
