#!/bin/bash
# Headline kernel: priority also raised around each node's (s, w) store (prio5, -DGP_SETPRIO=5) against
# the product (base), warm-up then four alternations, same box, P = 1e9.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_prio5}
mkdir -p $O
GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 60 > $O/warm.log 2>&1 || exit 1
for k in 1 2 3 4; do
  for v in base prio5; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 40 > $O/perf_${v}_$k.log 2>&1 || { tail -5 $O/perf_${v}_$k.log; exit 1; }
    echo "$v $k: $(grep -o '[0-9.]* ms/round kernel' $O/perf_${v}_$k.log | head -1)"
  done
done
