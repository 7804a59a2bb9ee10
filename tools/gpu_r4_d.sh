#!/bin/bash
# Round 4: the GPU test suite and the C3 sweep at the C4 shard sizes (tools/gpu_r4_check.sh), then the phase stamps
# of np8_wide_rows / np8_niw_post in the C5 conjugate sweep (experiment build).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4d}
mkdir -p $OUT
if [ -z "$SKIP_CHECK" ]; then OUT=$OUT/check bash tools/gpu_r4_check.sh || exit 1; fi
NP8_LIB_OVERRIDE=noparama_amd/lib/exp/niwt.so timeout -k 10 200 python -u bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 20 --cpu-seconds 0 > $OUT/niwt.json 2> $OUT/niwt.err || exit 1
grep "niw_post s=" $OUT/niwt.err | tail -6 || true
grep "wide_rows s=" $OUT/niwt.err | tail -9 || true
echo D_DONE
