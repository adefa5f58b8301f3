#!/bin/bash
# Build libcdr variants of replay.hip (name:flags pairs) into variants/libcdr_<name>.so,
# linking the other objects of the main build.  usage: tools/build_variants.sh "pf1:-DCDR_PF=1" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/cadence_amd/csrc"
OBJ="$ROOT/cadence_amd/csrc/build"
mkdir -p "$ROOT/variants"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I"$ROOT/include" --offload-arch=gfx950 $flags \
      -c "$ROOT/cadence_amd/csrc/replay.hip" -o "$ROOT/variants/replay_$name.o" &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/variants/libcdr_$name.so" \
      "$ROOT/variants/replay_$name.o" $(ls "$OBJ"/*.o | grep -v '/replay\.o$') -lpthread
  echo "built variants/libcdr_$name.so"
done
