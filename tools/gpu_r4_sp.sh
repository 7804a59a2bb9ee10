#!/bin/bash
# Round 4: the C3 assign without its hot-path spill -- GPU tests on the C3 path, WRITE_SIZE, and the driver's command.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4sp}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_fold.py tests/test_gpu_parity.py tests/test_gpu_fast_split.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B="bench.py --steps 40 --warmup 20 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o run -- python3 $B > $OUT/w.log 2>&1 || exit 1
python3 - <<PY
import csv, glob, collections
f = glob.glob("$OUT/w/**/run_counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "assign" in r["Kernel_Name"]:
        per[r["Kernel_Name"][:70]].append(float(r["Counter_Value"]))
for k, x in per.items():
    x.sort(); print(k, "n", len(x), "median WRITE_SIZE", x[len(x)//2])
PY
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-c5 > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1]); c=d['cold_start']; print('driver cmd', round(d['value']), 'sweeps/s; assign', round(d['roofline']['assign_ms_per_launch'] * 1e3, 2), 'us; cold', round(c['value']), 'mixed_ms', round(c['mixed']['ms_per_sweep'], 4))"
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5 > $OUT/s200.json 2> $OUT/s200.err || exit 1
python -c "import json; d=json.loads(open('$OUT/s200.json').read().strip().splitlines()[-1]); print('200 steps', round(d['value']), 'sweeps/s', round(d['ms_per_step'] * 1e3, 2), 'us/sweep')"
echo SP_DONE
