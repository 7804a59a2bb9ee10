export TMPDIR=/tmp
for v in base; do
  mkdir -p gpurun_out/pv/$v
  L=""; if [ $v != base ]; then L="NP8_LIB_OVERRIDE=$PWD/noparama_amd/lib/exp/$v.so"; fi
  env $L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv/$v -o run -- python3 bench.py --steps 40 --warmup 20 --cpu-seconds 0 --cold-sweeps 0 > gpurun_out/pv/$v.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv
for v in ("base",):
    for r in csv.DictReader(open(f"gpurun_out/pv/{v}/run_kernel_stats.csv")):
        print(v, r["Name"][:40], r["Calls"], r["AverageNs"])
PY
