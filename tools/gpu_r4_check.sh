#!/bin/bash
# Round-4 check (one GPU call): the GPU test suite, then the C3 sweep at the C4 shard sizes (local exchange and the
# one-rank RCCL path) and the default bench line.  Each step under its own time limit; the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4check}
mkdir -p $OUT
T=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
for n in ${SIZES:-1000000 125000}; do
  timeout -k 10 200 python -u bench.py $A --n $n > $OUT/local_$n.json 2> $OUT/local_$n.err || exit 1
  timeout -k 10 200 python -u bench.py $A --n $n --exchange rccl > $OUT/rccl_$n.json 2> $OUT/rccl_$n.err || exit 1
done
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), "sweeps/s", round(d["ms_per_step"] * 1e3, 2), "us/sweep, assign_us",
          round(d["roofline"]["assign_ms_per_launch"] * 1e3, 2))
PY
echo CHECK_DONE
