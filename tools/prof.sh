#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root): kernel trace + stats, then one PMC pass
# per TCC counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
B="bench.py --steps 40 --warmup 20 --cpu-seconds 0 --cold-sweeps 0 --no-c5 $BENCH_EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
echo PROF_DONE
