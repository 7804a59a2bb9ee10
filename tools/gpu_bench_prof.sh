#!/bin/bash
# One GPU call: a default bench line, then the profiling passes of tools/prof.sh into $OUT/prof.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err &&
bash tools/prof.sh $OUT/prof &&
echo GPU_BENCH_PROF_DONE
