#!/bin/bash
# One parameterised GPU recipe (replaces the per-experiment gpu_r4_*.sh one-offs).  Run on the GPU box from the repo
# root, e.g.  /usr/local/graft/bin/gpurun -- 'OUT=gpurun_out/x bash tools/gpu_job.sh tests smoke bench:c3:'
# Jobs (fields separated by ':', spaces inside a field written as ','):
#   tests[:<pytest -k expr>]        pytest -m gpu (one process, per-test timeout)
#   smoke                           __graft_entry__.smoke()
#   bench:<name>:<args>[:<env>]     python bench.py <args> > $OUT/<name>.json, one summary line
#   py:<name>:<script args>[:<env>] python <script args> > $OUT/<name>.out
#   cmd:<name>:<program args>       any program (a probe built in-tree) > $OUT/<name>.out
#   trace:<name>:<script args>      rocprofv3 --kernel-trace --stats of python <script args> -> $OUT/<name>/
#   pmc:<name>:<script args>        three rocprofv3 PMC passes (SQ issue/wait, FETCH_SIZE, WRITE_SIZE) -> $OUT/<name>/
# Every step has its own time limit; the first failing step ends the recipe (no GPU step after a failure).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/job}
mkdir -p "$OUT"
sp() { echo "${1//,/ }"; }
for job in "$@"; do
  IFS=':' read -r kind name args envs <<< "$job"
  A=$(sp "$args"); E=$(sp "$envs")
  case $kind in
    tests)
      if [ -n "$name" ]; then KA=(-k "$(sp "$name")"); else KA=(); fi
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" \
        > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
      tail -1 "$OUT/gpu_tests.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$OUT/smoke.log" 2>&1 \
        || { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    bench)
      env $E timeout -k 10 600 python -u bench.py $A > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
      python tools/bench_line.py "$OUT/$name.json" "$name" ;;
    py)
      env $E timeout -k 10 600 python -u $A > "$OUT/$name.out" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
      tail -3 "$OUT/$name.out" ;;
    cmd)
      timeout -k 10 300 $A > "$OUT/$name.out" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
      tail -3 "$OUT/$name.out" ;;
    trace)
      mkdir -p "$OUT/$name"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name/trace" -o run -- python3 $A \
        > "$OUT/$name/trace.log" 2>&1 || { tail -20 "$OUT/$name/trace.log"; exit 1; }
      python tools/trace_tail.py "$OUT/$name/trace" 0.5 "$OUT/$name/tail.json" | head -12 ;;
    pmc)
      mkdir -p "$OUT/$name"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name/trace" -o run -- python3 $A \
        > "$OUT/$name/trace.log" 2>&1 || exit 1
      timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/$name/sq" -o run -- python3 $A \
        > "$OUT/$name/sq.log" 2>&1 || exit 1
      timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$name/fetch" -o run -- python3 $A \
        > "$OUT/$name/fetch.log" 2>&1 || exit 1
      timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$name/write" -o run -- python3 $A \
        > "$OUT/$name/write.log" 2>&1 || exit 1
      echo "pmc $name done" ;;
    *) echo "unknown job $job"; exit 2 ;;
  esac
done
echo JOB_DONE
