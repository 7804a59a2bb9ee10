#!/bin/bash
# The round-end check on the final build: the -m gpu suite, smoke(), the default bench line and C5 niw_conjugate.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fc2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 200 python -u bench.py --config C5 --param-update niw_conjugate --steps 40 --warmup 10 --cpu-seconds 0 > $OUT/c5_conj.json 2> $OUT/c5_conj.err &&
echo FINAL_C_DONE
