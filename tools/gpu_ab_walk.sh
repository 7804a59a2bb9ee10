#!/bin/bash
# One GPU call: parity tests with the LDS-staged candidate walk (the default build), then the C3 bench with its
# cold / mixed legs for that build and for the v_readlane walk (noparama_amd/lib/exp/walk_readlane.so).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/walk}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-c5 > $OUT/lds.json 2> $OUT/lds.err &&
NP8_LIB_OVERRIDE=noparama_amd/lib/exp/walk_readlane.so timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-c5 > $OUT/readlane.json 2> $OUT/readlane.err &&
echo WALK_DONE
