set -o pipefail
mkdir -p gpurun_out/sub
for S in 1 4 8 16; do
  K=""; if [ $S -ge 16 ]; then K="--kcap 1024"; fi
  timeout -k 10 200 python -u bench.py --steps 200 --warmup 40 --cpu-seconds 0 --cold-sweeps 20 --substeps $S $K > gpurun_out/sub/s$S.json 2> gpurun_out/sub/s$S.err || exit 1
done
python - <<'PY'
import json
for S in (1,4,8,16):
    d=json.loads(open(f"gpurun_out/sub/s{S}.json").read().strip().splitlines()[-1])
    print(S, round(d["value"]), "sweeps/s assign_us", round(d["roofline"]["assign_ms_per_launch"]*1e3,1), "cold", round(d["cold_start"]["value"]), d["cold_start"]["K_per_sweep"][-1])
PY
