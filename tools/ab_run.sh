#!/bin/bash
# A/B timing of library variants on one GPU box (run there, from the repo root), interleaved R rounds:
#   OUT=gpurun_out/ab R=2 ARGS="--steps 200 --warmup 20" bash tools/ab_run.sh base=noparama_amd/lib/libnp8.so \
#       v1=noparama_amd/lib_exp/v1/libnp8.so
# Each run: bench.py (C3 warm state, no cold/C5/CPU legs unless ARGS asks) with NP8_LIB_OVERRIDE; one line per run.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ab}
R=${R:-2}
ARGS=${ARGS:-"--steps 200 --warmup 20"}
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for kv in "$@"; do
    name=${kv%%=*}; lib=${kv#*=}
    NP8_LIB_OVERRIDE=$lib timeout -k 10 300 python -u bench.py $ARGS --cold-sweeps 0 --cpu-seconds 0 --no-c5 \
      > "$OUT/$name.$r.json" 2> "$OUT/$name.$r.err" || { tail -20 "$OUT/$name.$r.err"; exit 1; }
    python tools/bench_line.py "$OUT/$name.$r.json" "$name.$r"
  done
done
echo AB_DONE
