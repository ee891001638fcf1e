#!/bin/bash
# Same-box A/B of the drop-in call rate (bench.py --dropin-only: FrameProcessor.__call__ per host frame, a fresh
# process each run), default vs each environment setting given, interleaved.
#   tools/ab_dropin.sh <tag> <rounds> "VAR=V [VAR=V..]" ...
set -e -o pipefail
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  timeout -k 10 200 python -u bench.py --dropin-only > "$OUT/default_$r.json" 2> "$OUT/default_$r.err"
  i=0
  for e in "$@"; do
    i=$((i + 1))
    env $e timeout -k 10 200 python -u bench.py --dropin-only > "$OUT/alt${i}_$r.json" 2> "$OUT/alt${i}_$r.err"
  done
done
i=0; for e in "$@"; do i=$((i + 1)); echo "alt$i = $e"; done
for f in "$OUT"/*.json; do
  echo "$f $(python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d.get('value'), d.get('ms_per_call'))")"
done
