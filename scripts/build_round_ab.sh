#!/bin/bash
# Same-box A/B libraries of the round kernels: gp_round.hip at a git revision (or the working
# tree) compiled into the experiments build, linked with the experiments objects of the other
# sources.  scripts/build_round_ab.sh <name> <rev|WORKTREE|file.hip>  ->  build/ablate/lib_<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2
make -s -C gossipprotocol_amd/csrc >/dev/null
mkdir -p build/ablate/src
src=build/ablate/src/gp_round_$name.hip
if [ "$rev" = WORKTREE ]; then cp gossipprotocol_amd/csrc/gp_round.hip $src; elif [ -f "$rev" ]; then cp "$rev" $src; else git show $rev:gossipprotocol_amd/csrc/gp_round.hip > $src; fi
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGP_EXPERIMENTS -Igossipprotocol_amd/csrc $EXTRA"
others=$(ls build/obj_exp/*.o | grep -v "/gp_round.o")
/opt/rocm/bin/hipcc $FLAGS -c $src -o build/ablate/gp_round_$name.o
/opt/rocm/bin/hipcc $FLAGS -shared -o build/ablate/lib_$name.so $others build/ablate/gp_round_$name.o -L/opt/rocm/lib -lrccl
echo build/ablate/lib_$name.so
