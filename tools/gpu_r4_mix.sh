#!/bin/bash
# Round 4: the mixed / cold legs of the default bench, A/B of the round-4 switches (conditional lists, folded check).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4mix}
mkdir -p $OUT
A="--steps 20 --warmup 5 --cpu-seconds 0 --no-c5"
for v in def lists nofold both; do
  case $v in def) E="";; lists) E="NP8_LISTS_ALWAYS=1";; nofold) E="NP8_NO_LLFOLD=1";; both) E="NP8_LISTS_ALWAYS=1 NP8_NO_LLFOLD=1";; esac
  env $E timeout -k 10 300 python -u bench.py $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); c=d['cold_start']; print('$v', 'warm', round(d['value']), 'cold', round(c['value']), 'mixed_ms', round(c['mixed']['ms_per_sweep'], 4))"
done
echo MIX_DONE
