#!/bin/bash
# same-box A/B of the headline: default vs the round-5 P2 forms off
set -e -o pipefail
OUT=gpurun_out/r05ab
mkdir -p $OUT
B="python -u bench.py --steps 20 --extras none --cpu-sample 0 --no-prof --no-ingest"
for r in 1 2; do
  timeout -k 10 200 $B > $OUT/on_$r.json 2> $OUT/on_$r.err
  VA_CONV3Q=0 VA_STEM_TAIL=0 timeout -k 10 200 $B > $OUT/off_$r.json 2> $OUT/off_$r.err
  VA_CONV3Q=0 VA_STEM_TAIL=0 VA_STEM=0 timeout -k 10 200 $B > $OUT/nostem_$r.json 2> $OUT/nostem_$r.err
done
for f in $OUT/*.json; do echo "$f $(python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"; done
