#!/bin/bash
# Build experiment variants of the push-sum column kernel (gp_pscol.hip with extra -D flags),
# each linked with the experiments objects of the other sources: build/ablate/lib_pc_<name>.so
set -e
cd "$(dirname "$0")/.."
make -s -C gossipprotocol_amd/csrc >/dev/null
mkdir -p build/ablate
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGP_EXPERIMENTS"
others=$(ls build/obj_exp/*.o | grep -v gp_pscol.o)
declare -A V=( [nr2m4]="-DGP_PC_NR=2 -DGP_PC_MINW=4 -DGP_PC_AHEAD=1" [nr4m3]="-DGP_PC_NR=4 -DGP_PC_MINW=3 -DGP_PC_AHEAD=1"
               [nr4m4]="-DGP_PC_NR=4 -DGP_PC_MINW=4 -DGP_PC_AHEAD=1" [nr2m5]="-DGP_PC_NR=2 -DGP_PC_MINW=5 -DGP_PC_AHEAD=1"
               [nr2a2]="-DGP_PC_NR=2 -DGP_PC_MINW=4 -DGP_PC_AHEAD=2" [nr4m3a2]="-DGP_PC_NR=4 -DGP_PC_MINW=3 -DGP_PC_AHEAD=2"
               [nr2a3]="-DGP_PC_NR=2 -DGP_PC_MINW=4 -DGP_PC_AHEAD=3" )
for v in ${ONLY:-${!V[@]}}; do
  /opt/rocm/bin/hipcc $FLAGS ${V[$v]} -c gossipprotocol_amd/csrc/gp_pscol.hip -o build/ablate/gp_pscol_$v.o &
done
wait
for v in ${ONLY:-${!V[@]}}; do
  /opt/rocm/bin/hipcc $FLAGS -shared -o build/ablate/lib_pc_$v.so $others build/ablate/gp_pscol_$v.o -L/opt/rocm/lib -lrccl
done
ls build/ablate/lib_pc_*.so
