#!/bin/bash
# C5 niw_conjugate kernel times per library variant (tools/build_variant.sh): one rocprofv3 kernel-trace
# pass of a short bench run each, into gpurun_out/c5v/<name>/; prints the parameter-update kernels.
# usage (GPU box): bash tools/c5_variants.sh base <variant>...   ("base" = the product library)
set -o pipefail
export TMPDIR=/tmp
ARGS=${C5_ARGS:-"--config C5 --param-update niw_conjugate --steps 20 --warmup 20 --cpu-seconds 0 --cold-sweeps 0"}
for v in "$@"; do
  out=gpurun_out/c5v/$v
  mkdir -p $out
  if [ "$v" = base ]; then unset NP8_LIB_OVERRIDE; else export NP8_LIB_OVERRIDE=$PWD/noparama_amd/lib/exp/$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 -u bench.py $ARGS \
    > $out/bench.json 2> $out/bench.err || exit 1
done
python3 - "$@" <<'PY'
import csv, glob, json, sys
for v in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/c5v/{v}/**/run_kernel_stats.csv", recursive=True)
    rows = {r["Name"]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f[0]))} if f else {}
    b = json.loads(open(f"gpurun_out/c5v/{v}/bench.json").read().strip().splitlines()[-1])
    sel = {k.split("(")[0].split("::")[-1][:40]: round(t, 1) for k, t in rows.items() if t > 20}
    print(v, round(b["value"], 1), "sweeps/s", sel)
PY
