#!/bin/bash
# One GPU call: parity tests touching the max-likelihood check, A/B of the reduce fused into np8_loglik
# (NP8_LLFUSE=0 = separate np8_loglik_reduce) at N = 125k and 1e6, then a kernel trace of the mixed regime.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ll}
mkdir -p $OUT
A="--steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_resume.py tests/test_gpu_rccl_one_rank.py tests/test_gpu_membertrix.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_on.json 2> $OUT/n125k_on.err &&
NP8_LLFUSE=0 timeout -k 10 120 python -u bench.py $A --n 125000 > $OUT/n125k_off.json 2> $OUT/n125k_off.err &&
timeout -k 10 120 python -u bench.py $A > $OUT/n1m_on.json 2> $OUT/n1m_on.err &&
NP8_LLFUSE=0 timeout -k 10 120 python -u bench.py $A > $OUT/n1m_off.json 2> $OUT/n1m_off.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/mixed -o run -- python3 tools/mixed_state.py 150 > $OUT/mixed.log 2>&1 &&
echo LL_DONE
