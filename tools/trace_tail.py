"""Per-kernel durations over the LAST part of a rocprofv3 kernel trace (the steady regime of a run whose first
dispatches are a different regime: the cold start before the mixed one, or the warm-up before a bench's timed
sweeps), plus the idle time between consecutive dispatches.
usage: python tools/trace_tail.py <dir with run_kernel_trace.csv> [tail_fraction=0.3] [json_out]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
paths = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
rows = []
for p in paths:
    for r in csv.DictReader(open(p)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
tail = rows[int(len(rows) * (1.0 - frac)):]
dur = defaultdict(list)
gaps = []
for k, (s, e, n) in enumerate(tail):
    dur[n].append(e - s)
    if k:
        gaps.append(s - tail[k - 1][1])
span = tail[-1][1] - tail[0][0] if tail else 0
out = {"dispatches": len(tail), "span_ns": span,
       "busy_ns": sum(e - s for s, e, _ in tail),
       "gap_ns_median": sorted(gaps)[len(gaps) // 2] if gaps else None,
       "kernels": {n: {"calls": len(v), "avg_ns": sum(v) / len(v), "total_ns": sum(v)}
                   for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))}}
for n, v in out["kernels"].items():
    print(f"{v['calls']:6d} {v['avg_ns'] / 1e3:9.2f} us avg {v['total_ns'] / 1e3:10.1f} us total  {n[:90]}")
print("dispatches", out["dispatches"], "span us", span / 1e3, "busy us", out["busy_ns"] / 1e3,
      "median gap us", (out["gap_ns_median"] or 0) / 1e3)
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
