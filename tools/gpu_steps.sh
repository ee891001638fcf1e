#!/bin/bash
# Runs GPU steps in order, each under its own time limit; a step that fails its checks (exit 1) lets the next
# one run, anything else (fault, abort, signal, time limit) ends the script there.
#   bash tools/gpu_steps.sh SECONDS LOGNAME -- cmd ... [:: SECONDS LOGNAME -- cmd ...]
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
  t=$1; log=$2; shift 3
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "::" ]; do cmd+=("$1"); shift; done
  [ "$1" = "::" ] && shift
  mkdir -p "$(dirname "gpurun_out/$log")"
  echo "== ${cmd[*]}  (limit ${t}s, log gpurun_out/$log)"
  timeout -k 10 "$t" "${cmd[@]}" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 4 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
