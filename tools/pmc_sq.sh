#!/bin/bash
# One SQ counter pass of the C3 bench (run on the GPU box from the repo root) per library variant:
#   bash tools/pmc_sq.sh OUTDIR name=lib.so [name=lib.so ...]
# then: python tools/pmc_sq_summary.py OUTDIR
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
B="bench.py --steps 40 --warmup 20 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
for kv in "$@"; do
  name=${kv%%=*}; lib=${kv#*=}
  NP8_LIB_OVERRIDE=$lib timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d "$OUT/$name" -o run -- python3 $B > "$OUT/$name.log" 2>&1 || exit 1
done
echo PMC_DONE
