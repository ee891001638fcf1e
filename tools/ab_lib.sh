#!/bin/bash
# Same-box A/B of the headline between this tree's libva355.so and a variant build of the same C-ABI
# (tools/build_variant.sh -> vision_assist_amd/libva355_<name>.so), runs interleaved; then the per-layer profile of each.
#   tools/ab_lib.sh <tag> <variant name> <rounds>
set -o pipefail
TAG=$1; V=$2; ROUNDS=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="python -u bench.py --steps 20 --warmup 5 --extras none --cpu-sample 0 --no-ingest"
for r in $(seq 1 "$ROUNDS"); do
  timeout -k 10 300 $B > "$OUT/cur_$r.json" 2> "$OUT/cur_$r.err" || exit 1
  VA355_LIB=$PWD/vision_assist_amd/libva355_$V.so timeout -k 10 300 $B > "$OUT/${V}_$r.json" 2> "$OUT/${V}_$r.err" || exit 1
done
timeout -k 10 300 python -u tools/seg_layer_profile.py --dtype f32 --batch 256 --iters 5 --json "$OUT/layers_cur.json" > "$OUT/layers_cur.log" 2>&1 || exit 1
VA355_LIB=$PWD/vision_assist_amd/libva355_$V.so timeout -k 10 300 python -u tools/seg_layer_profile.py --dtype f32 --batch 256 --iters 5 \
  --json "$OUT/layers_$V.json" > "$OUT/layers_$V.log" 2>&1 || exit 1
for f in "$OUT"/*_[0-9].json; do
  echo "$f $(python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['avg_launch_us'],d['roofline']['frac'])")"
done
