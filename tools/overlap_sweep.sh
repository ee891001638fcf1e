#!/bin/bash
# Headline overlap sweep (network streams x batches in flight x batch), two interleaved rounds, one box.
set -e -o pipefail
OUT=gpurun_out/${1:-overlap}
mkdir -p "$OUT"
B="python -u bench.py --steps 20 --extras none --cpu-sample 0 --no-prof --no-ingest"
for r in 1 2; do
  for cfg in "2 3 256" "3 3 256" "2 4 256" "3 4 256" "2 3 384" "3 4 384" "2 3 192"; do
    set -- $cfg
    timeout -k 10 200 $B --seg-streams $1 --pipelines $2 --batch $3 > "$OUT/s$1_p$2_b$3_$r.json" 2>/dev/null
  done
done
for f in "$OUT"/*.json; do
  echo "$f $(python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['value'])")"
done
