#!/bin/bash
# Build a variant of libqie.so with extra compile flags, for same-process A/B (tools/ab.py).
#   bash tools/build_variant.sh <name> [-DFLAG=V ...]   ->  tools/ab_build/<name>.so
# ONLY=<src> (e.g. ONLY=attention) recompiles just that source with the flags and links it with
# the main build's other objects (qwen_image_edit_streamdiffusion_amd/csrc/build/*.o).
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
OUT=tools/ab_build/$NAME
mkdir -p $OUT
MAIN=qwen_image_edit_streamdiffusion_amd/csrc/build
pids=()
for f in qwen_image_edit_streamdiffusion_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ -n "$ONLY" ] && [ "$b" != "$ONLY" ]; then cp $MAIN/$b.o $OUT/$b.o; continue; fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-inline-asm \
    ${QIE_VARIANT_BASEFLAGS--Xclang -target-feature -Xclang -packed-fp32-ops -ffp-contract=off} "$@" \
    -c $f -o $OUT/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "build of $NAME failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/ab_build/$NAME.so $OUT/*.o
rm -rf $OUT
echo tools/ab_build/$NAME.so
