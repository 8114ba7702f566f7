#!/bin/bash
# Build the experiments library of an earlier commit, for same-box A/B runs:
#   scripts/build_at.sh <commit> <out.so>      (CPU; the .so travels with the tree)
set -e
cd "$(dirname "$0")/.."
c=$1; out=$2
d=$(mktemp -d)
git archive "$c" gossipprotocol_amd/csrc include | tar -x -C "$d"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DGP_EXPERIMENTS"
objs=""
for f in "$d"/gossipprotocol_amd/csrc/*.hip; do
  o="$d/$(basename $f .hip).o"
  /opt/rocm/bin/hipcc $FLAGS -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
mkdir -p "$(dirname "$out")"
/opt/rocm/bin/hipcc $FLAGS -shared -o "$out" $objs -Wl,-soname,libgossip_hip_exp.so -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl
rm -rf "$d"
echo "$out"
