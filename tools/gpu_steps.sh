#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that ends in a fault, an abort,
# a segfault or a time limit (exit status >= 124, or 134 / 139) -- an ordinary failure (status 1-123, e.g.
# failing tests) does not stop the later steps.  Usage:
#   tools/gpu_steps.sh <outdir> "<seconds>:<name>:<command>" ...
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
worst=0
for spec in "$@"; do
  secs=${spec%%:*}
  rest=${spec#*:}
  name=${rest%%:*}
  cmd=${rest#*:}
  echo "[$(date +%T)] $name: $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -3 "$OUT/$name.log"
  [ $rc -gt $worst ] && worst=$rc
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
exit $worst
