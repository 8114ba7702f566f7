#!/bin/bash
# Same-box A/B libraries: one source (SRC, default gp_round) at a git revision, the working tree
# or a file, compiled into the experiments build (+ EXTRA flags) and linked with the experiments
# objects of the other sources.
#   [SRC=gp_col] [EXTRA=...] scripts/build_round_ab.sh <name> <rev|WORKTREE|file.hip>  ->  build/ablate/lib_<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2; S=${SRC:-gp_round}
make -s -C gossipprotocol_amd/csrc >/dev/null
mkdir -p build/ablate/src
src=build/ablate/src/${S}_$name.hip
if [ "$rev" = WORKTREE ]; then cp gossipprotocol_amd/csrc/$S.hip $src; elif [ -f "$rev" ]; then cp "$rev" $src; else git show $rev:gossipprotocol_amd/csrc/$S.hip > $src; fi
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGP_EXPERIMENTS -Igossipprotocol_amd/csrc"
others=$(ls build/obj_exp/*.o | grep -v "/$S.o")
/opt/rocm/bin/hipcc $FLAGS "${EXTRA_ARGS[@]}" $EXTRA -c $src -o build/ablate/${S}_$name.o
/opt/rocm/bin/hipcc $FLAGS -shared -o build/ablate/lib_$name.so $others build/ablate/${S}_$name.o -L/opt/rocm/lib -lrccl
echo build/ablate/lib_$name.so
