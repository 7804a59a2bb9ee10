"""Per-wave instruction counts of the C3 assign kernel from tools/pmc_sq.sh passes: python tools/pmc_sq_summary.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*", ""))):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    acc = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "np8_assign_fast<8, 3, 0, false, false>" not in k:
            continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    w = sum(acc["SQ_WAVES"].values())
    print(os.path.basename(d.rstrip("/")), {c: round(sum(v.values()) / max(w, 1), 1) for c, v in acc.items() if c != "SQ_WAVES"},
          "waves/launch", round(w / max(len(acc["SQ_WAVES"]), 1)))
