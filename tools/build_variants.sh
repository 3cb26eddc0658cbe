#!/bin/bash
# Build A/B variants of libtruncgptq.so that differ in one translation unit's
# -D switches (development tool; results in gptq-svd_amd/variants/, git-ignored
# .so files that travel to the GPU box).
#   tools/build_variants.sh bulge "TG_BULGE_SPLIT=0" "TG_BULGE_SPLIT=3" ...
# Each argument after the unit is one variant: space-separated NAME=VALUE defines.
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
PK=$HERE/gptq-svd_amd
UNIT=$1; shift
make -s -C "$PK" -j8
mkdir -p "$PK/variants" "$PK/build/var"
FLAGS="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -Wno-unused-result"
OTHERS=$(ls "$PK"/build/*.o | grep -v "/$UNIT.o")
i=0
for V in "$@"; do
  TAG=v$i
  DEFS=""
  for d in $V; do DEFS="$DEFS -D$d"; done
  /opt/rocm/bin/hipcc $FLAGS $DEFS -c "$PK/csrc/$UNIT.hip" -o "$PK/build/var/${UNIT}_$TAG.o" &
  i=$((i+1))
done
wait
i=0
for V in "$@"; do
  TAG=v$i
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PK/variants/lib_${UNIT}_$TAG.so" \
    $OTHERS "$PK/build/var/${UNIT}_$TAG.o"
  echo "$PK/variants/lib_${UNIT}_$TAG.so: $V"
  i=$((i+1))
done
