#!/bin/bash
# Headline kernel, s_setprio variants: none (prio0), the product (prio3), from the in-edge pass's start
# (prio4), priority 1 / 3 instead of 2 (prio3v1 / prio3v3); three alternations, same box, P = 1e9.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_prio3}
mkdir -p $O
for k in 1 2 3; do
  for v in prio0 prio3 prio4 prio3v1 prio3v3; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 40 > $O/perf_${v}_$k.log 2>&1 || { tail -5 $O/perf_${v}_$k.log; exit 1; }
    echo "$v $k: $(grep -o '[0-9.]* ms/round kernel' $O/perf_${v}_$k.log | head -1)"
  done
done
