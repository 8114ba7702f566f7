#!/bin/bash
# Build in-tree first (a stale .so once reached the box), then run one gpurun call:
#   scripts/gpurun.sh <timeout s> '<command>'
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C gossipprotocol_amd/csrc >/dev/null
make -s -C oracle >/dev/null
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
