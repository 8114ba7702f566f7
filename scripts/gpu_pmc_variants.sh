#!/bin/bash
# FETCH_SIZE and TCC hit/miss passes for round-kernel variants ("ENV=VAL,ENV=VAL" words in $VARIANTS).
export TMPDIR=/tmp
N=${N:-1000000000}; TOPO=${TOPO:-Imp3D}; ALG=${ALG:-push-sum}
i=0
for v in ${VARIANTS:-default}; do
  i=$((i+1))
  if [ "$v" = default ]; then envs=""; else envs="${v//,/ }"; fi
  mkdir -p gpurun_out/pmcv/v$i; echo "$v" > gpurun_out/pmcv/v$i/name.txt
  env $envs timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcv/v$i/f -o f -- python3 tools/perf_round.py $N $TOPO $ALG 10 > gpurun_out/pmcv/v$i/f.log 2>&1 || exit 1
  env $envs timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcv/v$i/h -o h -- python3 tools/perf_round.py $N $TOPO $ALG 10 > gpurun_out/pmcv/v$i/h.log 2>&1 || exit 1
done
