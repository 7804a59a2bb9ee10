#!/bin/bash
# One GPU call: the -m gpu suite, then A/B of the fused finalize + lists launch (np8_fin_prune; NP8_FINPRUNE=0 = two
# launches) on the C3 sweep at N = 125k and 1e6, then the default bench line.  Each GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/fp}
mkdir -p $OUT
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_on.json 2> $OUT/n125k_on.err &&
NP8_FINPRUNE=0 timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_off.json 2> $OUT/n125k_off.err &&
timeout -k 10 120 python -u bench.py $A --n 125000 --exchange rccl > $OUT/n125k_rccl.json 2> $OUT/n125k_rccl.err &&
timeout -k 10 120 python -u bench.py $A --n 500000 > $OUT/n500k_on.json 2> $OUT/n500k_on.err &&
timeout -k 10 120 python -u bench.py $A > $OUT/n1m_on.json 2> $OUT/n1m_on.err &&
NP8_FINPRUNE=0 timeout -k 10 120 python -u bench.py $A > $OUT/n1m_off.json 2> $OUT/n1m_off.err &&
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
echo FP_DONE
