#!/bin/bash
# C4 budget at HEAD (local and one-rank RCCL at 1e6 / 500k / 250k / 125k items), the default bench line, and the
# niw_post phase stamps of the C5 conjugate sweep (experiment build).
set -o pipefail
export TMPDIR=/tmp
bash tools/c4_budget.sh || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/c4/bench.json 2> gpurun_out/c4/bench.err || exit 1
NP8_LIB_OVERRIDE=noparama_amd/lib/exp/niwt.so timeout -k 10 200 python -u bench.py --config C5 --param-update niw_conjugate --steps 20 --warmup 20 --cpu-seconds 0 > gpurun_out/c4/niwt.json 2> gpurun_out/c4/niwt.err || exit 1
grep "niw_post s=" gpurun_out/c4/niwt.err | tail -8 || true
echo C4_DONE
