#!/bin/bash
# One GPU call: the default bench line, the C3 profile (tools/prof.sh) and the C5 profile
# (tools/prof_c5.sh) at the current build.  Each GPU step under its own limit, chained.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fa}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
bash tools/prof.sh $OUT/prof &&
bash tools/prof_c5.sh $OUT/prof_c5 &&
echo FINAL_A_DONE
