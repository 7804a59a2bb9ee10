#!/bin/bash
# One GPU call: the -m gpu suite, a default bench line, then the profiling passes (tools/prof.sh).
# Every GPU step runs under its own time limit; the steps are chained so that a failure stops the call.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
echo GPU_CHECK_DONE
