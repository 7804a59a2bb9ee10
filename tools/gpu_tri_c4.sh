#!/bin/bash
# One GPU call: the triadic parity tests and bench (merge bound), then a kernel trace of the C3 sweep on a
# 125k-item shard (the C4 per-rank floor).  Each GPU step under its own limit, chained.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tc4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_triadic.py tests/test_gpu_splitmerge.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --sampler triadic --steps 10 --warmup 2 --cpu-seconds 0 --cold-sweeps 0 --no-c5 > $OUT/tri.json 2> $OUT/tri.err &&
timeout -k 10 200 python -u bench.py --n 125000 --steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5 > $OUT/n125k.json 2> $OUT/n125k.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace125k -o run -- python3 bench.py --n 125000 --steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5 > $OUT/trace125k.log 2>&1 &&
echo TRI_C4_DONE
