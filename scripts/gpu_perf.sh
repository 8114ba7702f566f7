#!/bin/bash
# Steady-state round timing of variants given as "ENV=VAL[,ENV=VAL] ..." words in $VARIANTS; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${N:-1000000000}; TOPO=${TOPO:-Imp3D}; ALG=${ALG:-push-sum}; R=${R:-10}
for v in ${VARIANTS:-default}; do
  echo "== $v" >> gpurun_out/perf_v.log
  if [ "$v" = default ]; then envs=""; else envs="${v//,/ }"; fi
  env $envs timeout -k 10 300 python -u tools/perf_round.py $N $TOPO $ALG $R >> gpurun_out/perf_v.log 2>&1 || exit 1
done
