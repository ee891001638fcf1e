#!/bin/bash
# Build an alternative libva355 from a modified va_seg.hip for same-box A/B timing:
#   tools/build_variant.sh /tmp/va_seg_X.hip X [extra hipcc flags, e.g. -DCONV2_ABL=1]  ->  vision_assist_amd/libva355_X.so
# then on the GPU box: VA355_LIB=$PWD/vision_assist_amd/libva355_X.so python tools/seg_layer_profile.py
set -e
SEG=$1; NAME=$2; shift 2; EXTRA="$*"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/vision_assist_amd/csrc
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -I$CSRC -I$ROOT/include -mllvm -amdgpu-atomic-optimizer-strategy=None"
OBJS="va_nav.o va_c2f.o va_c2fb.o va_stem.o va_pw.o va_post.o va_contour.o va_fp8.o va_handle.o"
make -s -C "$CSRC" $OBJS
SRC=$CSRC/.variant_$NAME.hip  # next to the real source: relative includes resolve
cp "$SEG" "$SRC"
/opt/rocm/bin/hipcc $FLAGS $EXTRA -c "$SRC" -o "$CSRC/.variant_$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o "$ROOT/vision_assist_amd/libva355_$NAME.so" \
    $(for o in $OBJS; do echo "$CSRC/$o"; done) "$CSRC/.variant_$NAME.o"
rm -f "$SRC" "$CSRC/.variant_$NAME.o"
echo "built vision_assist_amd/libva355_$NAME.so"
