#!/bin/bash
# Same-box A/B of the headline (bench.py, extras off): interleaved runs of the default and of each environment
# setting given.   tools/ab_headline.sh <tag> <rounds> "VAR=V [VAR=V..]" ["VAR=V ..."] ...
set -e -o pipefail
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="python -u bench.py --steps 20 --extras none --cpu-sample 0 --no-prof --no-ingest"
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
  echo "$f $(python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
