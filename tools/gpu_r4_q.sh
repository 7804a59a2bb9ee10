#!/bin/bash
# Round 4: the driver's own commands at HEAD -- smoke(), then bench.py as the driver runs it (N=1, --steps 20
# --warmup 5, default legs), with the host split of the timed region.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4q}
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
NP8_BENCH_PHASES=1 timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
grep "timed region" $OUT/bench.err || true
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), 'sweeps/s', round(d['ms_per_step'] * 1e3, 2), 'us/sweep; assign', round(d['roofline']['assign_ms_per_launch'] * 1e3, 2), 'us; c5', {k: round(v['value']) for k, v in d['c5'].items() if isinstance(v, dict) and 'value' in v})"
echo Q_DONE
