#!/bin/bash
# CPU: experiments-build libraries that differ only in gp_fullbin.hip's -D knobs
# (build/ablate/lib_<name>.so); run the csrc Makefile first.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGP_EXPERIMENTS"
OTHERS=$(ls build/obj_exp/*.o | grep -v gp_fullbin.o)
build() {  # name flags...
  local name=$1; shift
  /opt/rocm/bin/hipcc $FLAGS "$@" -c -o build/ablate/gp_fullbin_$name.o gossipprotocol_amd/csrc/gp_fullbin.hip
  /opt/rocm/bin/hipcc $FLAGS -shared -o build/ablate/lib_$name.so $OTHERS build/ablate/gp_fullbin_$name.o -L/opt/rocm/lib -lrccl
}
for v in ${FB_VARIANTS:-"fbv1:-DGP_FB_V2=0" "fbv2:"}; do
  name=${v%%:*}; flags=${v#*:}
  build $name ${flags//,/ } &
done
wait
