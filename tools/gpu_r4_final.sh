#!/bin/bash
# Round 4 final check on a fresh box: the full GPU suite, smoke(), the driver's bench command (N=1, default legs),
# and the C5 conjugate line.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); c=d['cold_start']; print('bench', round(d['value']), 'sweeps/s', round(d['ms_per_step'] * 1e3, 2), 'us/sweep; assign', round(d['roofline']['assign_ms_per_launch'] * 1e3, 2), 'us; frac', round(d['roofline']['frac'], 3), '; cold', round(c['value']), 'mixed_ms', round(c['mixed']['ms_per_sweep'], 4), '; c5', {k: round(v['value']) for k, v in d['c5'].items() if isinstance(v, dict) and 'value' in v})"
echo FINAL_DONE
