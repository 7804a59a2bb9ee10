#!/bin/bash
# One GPU call: the -m gpu suite with the lists' first candidate block preloaded (prune_row)
# (noparama_amd/lib/exp/fin.so), then A/B against the current build at N = 125k and 1e6 (twice each).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prn}
mkdir -p $OUT
L=noparama_amd/lib/exp/fin.so
A="--steps 300 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
NP8_LIB_OVERRIDE=$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
for k in 1 2; do
  NP8_LIB_OVERRIDE=$L timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_fin_$k.json 2> $OUT/e1 &&
  timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_cur_$k.json 2> $OUT/e2 &&
  NP8_LIB_OVERRIDE=$L timeout -k 10 120 python -u bench.py $A > $OUT/n1m_fin_$k.json 2> $OUT/e3 &&
  timeout -k 10 120 python -u bench.py $A > $OUT/n1m_cur_$k.json 2> $OUT/e4 || exit 1
done &&
echo FIN_DONE
