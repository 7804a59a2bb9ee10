#!/bin/bash
# C5 profile (run on the GPU box from the repo root): kernel trace + stats, HBM bytes (separate
# FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md "HBM"), and an SQ pass for issue/MFMA utilisation.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_c5}
mkdir -p $OUT
B="bench.py --config C5 --steps 10 --warmup 5 --cpu-seconds 0 $BENCH_EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $OUT/sq2 -o run -- python3 $B > $OUT/sq2.log 2>&1
echo PROF_DONE
