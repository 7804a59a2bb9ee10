#!/bin/bash
# One-GPU measurements behind DESIGN.md §6's multi-GPU budget: the C3 sweep on shards of 1e6/2, /4, /8 items
# (local exchange) and through a one-rank RCCL communicator (the sharded code path: staging, np8_req_select,
# ncclAllGather, finalize over the gathered record), plus C2.  JSON lines into gpurun_out/c4/.
set -o pipefail
mkdir -p gpurun_out/c4
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
for n in 1000000 500000 250000 125000; do
  timeout -k 10 200 python -u bench.py $A --n $n > gpurun_out/c4/local_$n.json 2> gpurun_out/c4/local_$n.err || exit 1
  timeout -k 10 200 python -u bench.py $A --n $n --exchange rccl > gpurun_out/c4/rccl_$n.json 2> gpurun_out/c4/rccl_$n.err || exit 1
done
timeout -k 10 200 python -u bench.py $A --n 100000 --d 2 --k 10 --config C2 > gpurun_out/c4/c2.json 2> gpurun_out/c4/c2.err || exit 1
python - <<'PY'
import json
for n in (1000000, 500000, 250000, 125000):
    for v in ("local", "rccl"):
        d = json.loads(open(f"gpurun_out/c4/{v}_{n}.json").read().strip().splitlines()[-1])
        print(n, v, round(d["value"]), "sweeps/s", round(d["ms_per_step"] * 1e3, 1), "us/sweep, assign_us",
              round(d["roofline"]["assign_ms_per_launch"] * 1e3, 1))
d = json.loads(open("gpurun_out/c4/c2.json").read().strip().splitlines()[-1])
print("C2", round(d["value"]), "sweeps/s", round(d["ms_per_step"] * 1e3, 1), "us/sweep")
PY
