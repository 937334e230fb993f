#!/usr/bin/env bash
# Run GPU steps in order under per-step time limits, logging each to gpurun_out/<tag>/<name>.log.
# Usage: tools/gpu_steps.sh <tag> "<name>|<timeout_s>|<command>" ...
# A step that ends in a fault, abort, segfault or time limit (exit >= 124, 134, 139) ends the run there: no
# further GPU step is started after a crash (test failures, exit 1, do not stop the run).
set -u
tag=$1; shift
out="gpurun_out/$tag"; mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "[gpu_steps] $name (limit ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $name rc=$rc in $(( $(date +%s) - start ))s"; tail -n 5 "$out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "[gpu_steps] stopping after $name"; exit $rc; fi
done
