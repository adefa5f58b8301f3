#!/bin/bash
# A/B builds: variants/libcdr_<name>.so = libcdr.so with replay.hip compiled under extra
# -D flags (load with CDR_LIB=variants/libcdr_<name>.so).  usage: tools/build_variant.sh <name> -DX=1 ...
set -e
name=$1; shift
cd "$(dirname "$0")/.."
make -s -C cadence_amd/csrc -j8
mkdir -p variants
objs=$(ls cadence_amd/csrc/build/*.o | grep -v '/replay.o$')
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Iinclude -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 \
  -munsafe-fp-atomics "$@" -c -o variants/replay_$name.o cadence_amd/csrc/replay.hip
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libcdr_$name.so variants/replay_$name.o $objs -lpthread
echo variants/libcdr_$name.so
