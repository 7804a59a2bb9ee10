"""One summary line of a bench.py JSON output (tools/gpu_job.sh).  usage: python tools/bench_line.py <file> [name]"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
name = sys.argv[2] if len(sys.argv) > 2 else ""
ro = d.get("roofline") or {}
out = [name, d.get("config", {}).get("workload", "")[:30], f"{d['value']:.0f} {d['unit']}",
       f"{d['ms_per_step'] * 1e3:.2f} us/step"]
if ro.get("assign_ms_per_launch"):
    out.append(f"assign {ro['assign_ms_per_launch'] * 1e3:.2f} us frac {ro.get('frac', 0):.3f}")
c = d.get("cold_start")
if isinstance(c, dict) and "value" in c:
    out.append(f"cold {c['value']:.0f}")
    if isinstance(c.get("mixed"), dict):
        out.append(f"mixed {c['mixed']['ms_per_sweep'] * 1e3:.1f} us")
sv = d.get("survey_state")
if isinstance(sv, dict) and "ms_per_sweep" in sv:
    out.append(f"survey {sv['ms_per_sweep'] * 1e3:.1f} us K {sv['K_final']}")
c5 = d.get("c5")
if isinstance(c5, dict):
    out.append("c5 " + " ".join(f"{k}={v['value']:.0f}" for k, v in c5.items() if isinstance(v, dict) and "value" in v))
print(" | ".join(out))
