#!/bin/bash
# Round 4: WRITE_SIZE of the C3 assign with and without the folded max-likelihood check (NP8_NO_LLFOLD=1).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r4w}
mkdir -p $OUT
B="bench.py --steps 40 --warmup 20 --cpu-seconds 0 --cold-sweeps 0 --no-c5"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/def -o run -- python3 $B > $OUT/def.log 2>&1 || exit 1
NP8_NO_LLFOLD=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/nofold -o run -- python3 $B > $OUT/nofold.log 2>&1 || exit 1
python3 - <<PY
import csv, glob, collections
for v in ["def", "nofold"]:
    f = glob.glob("$OUT/%s/**/run_counter_collection.csv" % v, recursive=True)[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "assign" in r["Kernel_Name"]:
            per[r["Kernel_Name"][:70]].append(float(r["Counter_Value"]))
    for k, x in per.items():
        x.sort()
        print(v, k, "n", len(x), "min", x[0], "median", x[len(x)//2], "max", x[-1])
PY
echo W_DONE
