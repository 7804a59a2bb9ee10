"""Condense a tools/prof.sh output directory into profiles/<tag>_*.{csv,json}.

traffic per launch follows MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
usage: python tools/summarize_profile.py gpurun_out/prof_r01 r01
"""
import csv
import json
import os
import shutil
import subprocess
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))

agg = defaultdict(list)
for sub in ("fetch", "write", "sq", "sq2"):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
per_kernel = defaultdict(dict)
for (k, c), v in agg.items():
    per_kernel[k][c] = {"launches": len(v), "mean": sum(v) / len(v)}
out = {"source": src, "counters": per_kernel}
# the assign step: np8_assign_fast + np8_assign_queue (C3, launched once each per step), np8_assign_wide (C5) or
# np8_assign; counting instances (template flag true) run outside the timed sweeps and are left out
def counting(k):  # the executed-work counting instances (COUNT = true) run outside the timed sweeps
    return "assign_wide" not in k and ((("true>" in k) and ("false, true>" not in k)) or (", true, false>" in k))


assign = [k for k in per_kernel if "np8_assign" in k and not counting(k) and "matrix" not in k]
assign.sort(key=lambda k: -per_kernel[k].get("SQ_WAVES", per_kernel[k].get("FETCH_SIZE", {})).get("launches", 0))
if assign:
    a = per_kernel[assign[0]]
    nl = a.get("FETCH_SIZE", {}).get("launches")
    step = [k for k in assign if per_kernel[k].get("FETCH_SIZE", {}).get("launches") == nl]
    out["assign_step_kernels"] = step
    fetch = sum(per_kernel[k].get("FETCH_SIZE", {}).get("mean", 0.0) for k in step)
    write = sum(per_kernel[k].get("WRITE_SIZE", {}).get("mean", 0.0) for k in step)
    if nl:
        out["assign_bytes_per_launch"] = (2.0 * fetch + write) * 1024.0
        out["assign_fetch_bytes_per_launch"] = 2.0 * fetch * 1024.0
        out["assign_write_bytes_per_launch"] = write * 1024.0
    if "SQ_INSTS_VALU" in a and "SQ_WAVES" in a:
        # SQ_INSTS_VALU counts wave-instructions; one item per lane, so this is also the VALU instruction
        # count of one item's lane
        out["assign_valu_insts_per_wave"] = a["SQ_INSTS_VALU"]["mean"] / a["SQ_WAVES"]["mean"]
    if "SQ_ACTIVE_INST_VALU" in a and "GRBM_GUI_ACTIVE" in a:
        # VALU issue utilisation (MI355X_MICROARCH.md counter units): SQ_ACTIVE_INST_VALU is summed over
        # waves in quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
        cyc = a["GRBM_GUI_ACTIVE"]["mean"] / 8.0
        out["assign_valu_issue_frac"] = 4.0 * a["SQ_ACTIVE_INST_VALU"]["mean"] / (1024.0 * cyc)
    if "SQ_WAIT_ANY" in a and "SQ_WAVE_CYCLES" in a:
        out["assign_wait_any_frac"] = a["SQ_WAIT_ANY"]["mean"] / a["SQ_WAVE_CYCLES"]["mean"]
try:
    commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                            text=True).stdout.strip()
except Exception:
    commit = None
out["commit"] = f"profiled at {commit}" if commit else None
json.dump(out, open(os.path.join(dst, f"{tag}_counters.json"), "w"), indent=1)
json.dump({"assign_bytes_per_launch": out.get("assign_bytes_per_launch"), "source": f"profiles/{tag}_counters.json",
           "commit": out["commit"]},
          open(os.path.join(dst, f"traffic_{tag}.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "counters"}, indent=1))
