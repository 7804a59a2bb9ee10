#!/bin/bash
# Round 4: PMC counters of np8_assign_wide in the C5 frozen and niw_conjugate sweeps.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4n}
mkdir -p $OUT
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
P2="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_SMEM"
for pu in frozen niw_conjugate; do
  B="bench.py --config C5 --param-update $pu --steps 5 --warmup 5 --cpu-seconds 0 --cold-sweeps 0"
  timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d $OUT/${pu}_1 -o run -- python3 $B > $OUT/${pu}_1.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc $P2 --output-format csv -d $OUT/${pu}_2 -o run -- python3 $B > $OUT/${pu}_2.log 2>&1 || exit 1
done
python3 - <<PY
import csv, glob, collections
for pu in ["frozen", "niw_conjugate"]:
    acc = collections.defaultdict(list)
    for p in (1, 2):
        for f in glob.glob("$OUT/%s_%d/**/run_counter_collection.csv" % (pu, p), recursive=True):
            for r in csv.DictReader(open(f)):
                if "assign_wide" in r["Kernel_Name"]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(pu, {k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
PY
echo N_DONE
