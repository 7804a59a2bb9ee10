#!/bin/bash
# PMC passes on the mixed regime (tools/mixed_state.py): HBM bytes and the SQ issue/wait counters of the assign
# kernel over sweeps 0..79 after init_random(20) (the later dispatches are the mixed regime).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_mixed}
mkdir -p $OUT
B="tools/mixed_state.py 80"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1
echo PROF_DONE
