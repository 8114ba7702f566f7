#!/bin/bash
# Tile-walk A/B: parity of the tile kernels under the x-window walk, then
# steady-state round time per walk / window width; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
GP_WALK=2 GP_WX=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_walk2.log 2>&1 || exit 1
for cfg in "0 40" "2 8" "2 20" "2 40" "2 125"; do
  set -- $cfg
  echo "== walk $1 wx $2" >> gpurun_out/perf_walk.log
  GP_WALK=$1 GP_WX=$2 timeout -k 10 200 python -u tools/perf_round.py ${N:-1000000000} Imp3D push-sum 10 >> gpurun_out/perf_walk.log 2>&1 || exit 1
done
for cfg in "0 40" "2 20"; do
  set -- $cfg
  echo "== gossip walk $1 wx $2" >> gpurun_out/perf_walk.log
  GP_KERNEL=tile GP_WALK=$1 GP_WX=$2 timeout -k 10 200 python -u tools/perf_round.py 100000000 Imp3D gossip 20 >> gpurun_out/perf_walk.log 2>&1 || exit 1
done
