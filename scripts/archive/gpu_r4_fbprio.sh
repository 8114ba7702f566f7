#!/bin/bash
# C4 fused fold / split priority, on a warm GPU: f0 = product settings, f2 = the fold's tile loads at
# raised priority (-DGP_FB_PRIO=2), f1 = fold + split loads and stores (-DGP_FB_PRIO=1); a 300-round
# warm-up first, then four alternations, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_fbprio}
mkdir -p $O
GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_f0.so timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 300 > $O/warm.log 2>&1 || { tail -5 $O/warm.log; exit 1; }
tail -1 $O/warm.log
for k in 1 2 3 4; do
  for v in f0 f2 f1; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 100 > $O/c4_${v}_$k.log 2>&1 || { tail -5 $O/c4_${v}_$k.log; exit 1; }
    echo "$v $k: $(grep -o '[0-9.]* ms/round kernel' $O/c4_${v}_$k.log | head -1)"
  done
done
