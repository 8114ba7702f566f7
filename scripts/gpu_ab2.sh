#!/bin/bash
# A/B of the product library against build/exp/lib_prev.so on one box, alternating; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab2.log
for i in 1 2; do
  for v in prev cur; do
    if [ $v = prev ]; then export GOSSIP_HIP_LIB_EXPERIMENT=build/exp/lib_prev.so; else unset GOSSIP_HIP_LIB_EXPERIMENT; fi
    echo "== $v $(timeout -k 10 200 python -u tools/perf_round.py ${N:-1000000000} ${TOPO:-Imp3D} push-sum 10 | grep -o 'k_ps_tile<[A-Z0-9]*>: [0-9.]* ms')" >> gpurun_out/ab2.log || exit 1
  done
done
cat gpurun_out/ab2.log
