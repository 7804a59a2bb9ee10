#!/bin/bash
# One GPU call: the wide-path tests with the eigenvalue bracket stopped at 5% width (noparama_amd/lib/exp/lam5.so),
# then C5 with niw_conjugate and frozen for that build and for the default (2%).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/lam}
mkdir -p $OUT
L=noparama_amd/lib/exp/lam5.so
A="--config C5 --steps 40 --warmup 10 --cpu-seconds 0"
NP8_LIB_OVERRIDE=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_niw.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
NP8_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py $A --param-update niw_conjugate > $OUT/conj_lam5.json 2> $OUT/conj_lam5.err &&
timeout -k 10 200 python -u bench.py $A --param-update niw_conjugate > $OUT/conj_lam2.json 2> $OUT/conj_lam2.err &&
NP8_LIB_OVERRIDE=$L timeout -k 10 200 python -u bench.py $A > $OUT/frozen_lam5.json 2> $OUT/frozen_lam5.err &&
timeout -k 10 200 python -u bench.py $A > $OUT/frozen_lam2.json 2> $OUT/frozen_lam2.err &&
echo LAM_DONE
