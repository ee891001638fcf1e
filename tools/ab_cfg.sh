#!/bin/bash
# Same-box A/B of bench.py argument sets (each a quoted string), run interleaved round by round; prints value and
# ms_per_step per run.   tools/ab_cfg.sh <tag> <rounds> "<args A>" "<args B>" ...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for a in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python -u bench.py $a > "$OUT/v${i}_$r.json" 2> "$OUT/v${i}_$r.err" || { echo "v$i round $r failed"; exit 1; }
  done
done
i=0; for a in "$@"; do i=$((i + 1)); echo "v$i = $a"; done
for f in "$OUT"/v*.json; do
  echo "$f $(python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'))")"
done
