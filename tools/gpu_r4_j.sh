#!/bin/bash
# Round 4: PMC counters of np8_assign_wide (C5 frozen), the old fp32 screen (lib/exp/oldscreen.so) against the
# working tree's bf16 screen.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4j}
mkdir -p $OUT
B="bench.py --config C5 --steps 5 --warmup 5 --cpu-seconds 0 --cold-sweeps 0"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
for v in old cur; do
  if [ $v = old ]; then L=noparama_amd/lib/exp/oldscreen.so; else L=noparama_amd/lib/libnp8.so; fi
  NP8_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/$v -o run -- python3 $B > $OUT/$v.log 2>&1 || exit 1
done
python3 - <<PY
import csv, glob, collections
for v in ["old", "cur"]:
    f = glob.glob("$OUT/%s/**/run_counter_collection.csv" % v, recursive=True)
    if not f: print(v, "no csv"); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "assign_wide" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in acc.items()})
PY
echo J_DONE
