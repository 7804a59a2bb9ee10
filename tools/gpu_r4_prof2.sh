#!/bin/bash
# Round 4 profiles at the final build: C3 (prof.sh) and the mixed regime (prof_mixed.sh).
set -o pipefail
export TMPDIR=/tmp
bash tools/prof.sh gpurun_out/prof_r04b || exit 1
bash tools/prof_mixed.sh gpurun_out/prof_r04b_mixed || exit 1
echo PROF2_DONE
