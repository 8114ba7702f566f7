#!/bin/bash
# Build an experiments-build variant library: one source recompiled with extra -D flags,
# linked with the experiments objects of the other sources.
#   scripts/build_variant.sh <name> <source.hip> [-DFLAG=V ...]  ->  build/ablate/lib_<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
make -s -C gossipprotocol_amd/csrc >/dev/null
mkdir -p build/ablate
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGP_EXPERIMENTS"
base=$(basename "$src" .hip)
others=$(ls build/obj_exp/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc $FLAGS "$@" -c gossipprotocol_amd/csrc/$src -o build/ablate/${base}_$name.o
/opt/rocm/bin/hipcc $FLAGS -shared -o build/ablate/lib_$name.so $others build/ablate/${base}_$name.o -L/opt/rocm/lib -lrccl
echo build/ablate/lib_$name.so
