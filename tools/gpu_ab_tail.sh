#!/bin/bash
# One GPU call: the -m gpu suite with the one-workgroup tail (NP8_FUSE=1: finalize + lists in one launch on the
# sweeps that do not gather radii), then its A/B against separate launches at N = 125k and 1e6.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/tail}
mkdir -p $OUT
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
NP8_FUSE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
NP8_FUSE=1 timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_on.json 2> $OUT/n125k_on.err &&
timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_off.json 2> $OUT/n125k_off.err &&
NP8_FUSE=1 timeout -k 10 120 python -u bench.py $A > $OUT/n1m_on.json 2> $OUT/n1m_on.err &&
timeout -k 10 120 python -u bench.py $A > $OUT/n1m_off.json 2> $OUT/n1m_off.err &&
NP8_FUSE=1 timeout -k 10 120 python -u bench.py $A --n 500000 > $OUT/n500k_on.json 2> $OUT/n500k_on.err &&
NP8_FUSE=1 timeout -k 10 120 python -u bench.py $A --n 125000 --exchange rccl > $OUT/n125k_rccl_on.json 2> $OUT/n125k_rccl_on.err &&
NP8_FUSE=1 timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-c5 > $OUT/full_on.json 2> $OUT/full_on.err &&
echo TAIL_DONE
