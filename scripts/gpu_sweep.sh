#!/bin/bash
# Per-round kernel time across populations (tile kernel, per-round launches); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-"1000000 3D" "8000000 3D" "27000000 3D" "64000000 3D" "125000000 3D" "8000000 Imp3D"}; do
  set -- $cfg
  timeout -k 10 120 python -u tools/perf_round.py $1 $2 push-sum ${R:-50} || exit 1
done
