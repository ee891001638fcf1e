#!/bin/bash
# Same-box A/B of the bf16 extra (bench.py --extras bf16; headline steps cut to 3): interleaved runs of the default
# and of each environment setting given.   tools/ab_bf16.sh <tag> <rounds> "VAR=V [VAR=V..]" ...
set -e -o pipefail
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="python -u bench.py --steps 3 --warmup 1 --extras bf16 --cpu-sample 0 --no-prof --no-ingest"
for r in $(seq 1 "$ROUNDS"); do
  timeout -k 10 200 $B > "$OUT/default_$r.json" 2> "$OUT/default_$r.err"
  i=0
  for e in "$@"; do
    i=$((i + 1))
    env $e timeout -k 10 200 $B > "$OUT/alt${i}_$r.json" 2> "$OUT/alt${i}_$r.err"
  done
done
i=0; for e in "$@"; do i=$((i + 1)); echo "alt$i = $e"; done
for f in "$OUT"/*.json; do
  echo "$f $(python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d['extras']['bf16'];print(c['value'],c.get('ms_per_step'))")"
done
