#!/bin/bash
# Runs GPU steps one after another, each under its own time limit; a step that ends in a fault, abort,
# segfault or time limit stops the chain (test failures, exit 1, do not).
# usage: tools/gpu_steps.sh "<seconds> <command>" ...
mkdir -p gpurun_out
n=0
for step in "$@"; do
  n=$((n + 1))
  secs=${step%% *}
  cmd=${step#* }
  echo "[step $n] ($secs s) $cmd"
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "[step $n] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
