#!/bin/bash
# Same-box A/B of the C4 extra (bench.py --extras c4; headline steps cut to 3): interleaved runs of the default and of
# each setting given -- environment assignments, optionally followed by ':: <extra bench.py arguments>'.
#   tools/ab_c4.sh <tag> <rounds> "VAR=V [VAR=V..]" "GPU_MAX_HW_QUEUES=8 :: --c4-seg-streams 4" ...
set -e -o pipefail
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="python -u bench.py --steps 3 --warmup 1 --extras c4 --cpu-sample 0 --no-prof --no-ingest"
for r in $(seq 1 "$ROUNDS"); do
  timeout -k 10 200 $B > "$OUT/default_$r.json" 2> "$OUT/default_$r.err"
  i=0
  for e in "$@"; do
    i=$((i + 1))
    ev=${e%%::*}; ar=""
    [[ "$e" == *::* ]] && ar=${e#*::}
    env $ev timeout -k 10 200 $B $ar > "$OUT/alt${i}_$r.json" 2> "$OUT/alt${i}_$r.err"
  done
done
i=0; for e in "$@"; do i=$((i + 1)); echo "alt$i = $e"; done
for f in "$OUT"/*.json; do
  echo "$f $(python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);c=d['extras']['c4'];print(c['value'],c['ms_per_step'])")"
done
