#!/bin/bash
# Round close variants (GP_FUSE 0 separate finalize, 1 single-word fused, 2 sharded fused) x grid; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-"1000000 3D" "8000000 3D" "27000000 Imp3D" "125000000 3D" "1000000000 Imp3D"}; do
  set -- $cfg
  for v in ${VARS:-"GP_FUSE=1" "GP_FUSE=0" "GP_FUSE=2" "GP_FUSE=2 GP_GRID=5120" "GP_FUSE=0 GP_GRID=5120"}; do
    echo "== $1 $2 $v"
    env GP_EXP=1 GP_PERSIST=0 $v timeout -k 10 180 python -u tools/perf_round.py $1 $2 push-sum ${R:-20} || exit 1
  done
done
