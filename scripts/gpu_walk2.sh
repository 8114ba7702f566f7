#!/bin/bash
# Tile walk / window width sweep on the headline config; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/perf_walk.log
for cfg in ${CFGS:-"0 1" "2 8" "2 16"}; do
  set -- $cfg
  echo "== walk $1 wx $2" >> gpurun_out/perf_walk.log
  GP_WALK=$1 GP_WX=$2 timeout -k 10 200 python -u tools/perf_round.py 1000000000 Imp3D push-sum 10 >> gpurun_out/perf_walk.log 2>&1 || exit 1
done
cat gpurun_out/perf_walk.log
