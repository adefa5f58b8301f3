#!/bin/bash
# gfx950 disassembly of one kernel source (device-only compile with libcdr's flags) into
# /tmp/<name>.s, with a count of the instruction kinds worth watching (lane shuffles through
# LDS, DPP moves, readlanes) and a check that no scalar-cache store / atomic was emitted.
# usage: tools/isa.sh [replay.hip] [-DX=1 ...]
set -e
cd "$(dirname "$0")/../cadence_amd/csrc"
src=${1:-replay.hip}; shift || true
name=$(basename $src .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../../include -Wno-unused-function -Wno-unused-variable \
  --offload-arch=gfx950 -munsafe-fp-atomics --cuda-device-only "$@" -c -o /tmp/$name.dev.o $src
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/$name.dev.o \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/$name.co
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn /tmp/$name.co > /tmp/$name.s
echo "ds_bpermute $(grep -c ds_bpermute /tmp/$name.s || true)  dpp $(grep -c _dpp /tmp/$name.s || true)  readlane $(grep -c v_readlane /tmp/$name.s || true)"
bad=$(grep -cE "s_(store|atomic|buffer_store|buffer_atomic|dcache_wb|dcache_discard)" /tmp/$name.s || true)
echo "scalar-cache writes: $bad"
[ "$bad" = 0 ]
