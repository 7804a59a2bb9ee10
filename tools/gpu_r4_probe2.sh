#!/bin/bash
# Round-4 probe: the GPU tests, the C3 sweep at 125k and 1e6 items (default build), and the per-wave phase stamps
# of np8_assign_fast (clock build) at both sizes.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4p2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
for n in 125000 1000000; do
  timeout -k 10 200 python -u bench.py $A --n $n > $OUT/local_$n.json 2> $OUT/local_$n.err || exit 1
  NP8_LIB_OVERRIDE=noparama_amd/lib/exp/clk.so timeout -k 10 180 python -u tools/clocks.py $n warm > $OUT/clk_$n.json 2> $OUT/clk_$n.err || exit 1
done
python - <<PY
import json, glob
for f in sorted(glob.glob("$OUT/local_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), "sweeps/s", round(d["ms_per_step"] * 1e3, 2), "us/sweep, assign_us",
          round(d["roofline"]["assign_ms_per_launch"] * 1e3, 2))
for f in sorted(glob.glob("$OUT/clk_*.json")):
    d = json.load(open(f))
    print(f, "span", round(d["launch_span_us"], 2), "lat", round(d["wave_latency_us_mean"], 2), {k: round(v, 2) for k, v in d["phase_us_mean"].items()})
PY
echo PROBE2_DONE
