#!/bin/bash
# A/B of changes switched by environment variables: C3 bench lines at N = 1e6 and N = 125000, the default build
# and once per variable given set to 1 (usage: tools/ab_env.sh VAR...), JSON lines into gpurun_out/abe/.
set -o pipefail
mkdir -p gpurun_out/abe
A=${AB_ARGS:-"--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"}
for n in 1000000 125000; do
  for v in base "$@"; do
    if [ "$v" = base ]; then E=""; else E="$v=1"; fi
    env $E timeout -k 10 200 python -u bench.py $A --n $n > gpurun_out/abe/${v}_$n.json 2> gpurun_out/abe/${v}_$n.err || exit 1
  done
done
python - base "$@" <<'PY'
import json, sys
for n in (1000000, 125000):
    for v in sys.argv[1:]:
        d = json.loads(open(f"gpurun_out/abe/{v}_{n}.json").read().strip().splitlines()[-1])
        print(n, v, round(d["value"]), "sweeps/s", round(d["ms_per_step"] * 1e3, 1), "us/sweep, assign_us",
              round(d["roofline"]["assign_ms_per_launch"] * 1e3, 1))
PY
