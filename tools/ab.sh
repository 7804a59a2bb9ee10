#!/bin/bash
# A/B run on the GPU box: the C3 bench line (no CPU baseline, no cold leg) for the product library and
# for each variant library given (tools/build_variant.sh), one JSON line each into gpurun_out/ab/.
set -o pipefail
mkdir -p gpurun_out/ab
ARGS=${AB_ARGS:-"--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"}
timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/ab/base.json 2> gpurun_out/ab/base.err || exit 1
for v in "$@"; do
  NP8_LIB_OVERRIDE=$PWD/noparama_amd/lib/exp/$v.so timeout -k 10 200 python -u bench.py $ARGS \
    > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
done
python - "$@" <<'PY'
import json, sys
for v in ["base"] + sys.argv[1:]:
    d = json.loads(open(f"gpurun_out/ab/{v}.json").read().strip().splitlines()[-1])
    print(v, round(d["value"]), "sweeps/s", "assign_us", round(d["roofline"]["assign_ms_per_launch"] * 1e3, 1))
PY
