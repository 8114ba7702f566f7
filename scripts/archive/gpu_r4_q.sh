#!/bin/bash
# q1 = the fold's tile loads at raised priority (-DGP_FB_PRIO=2) and the column kernel at priority 1
# instead of 2 (-DGP_COL_PRIO_VAL=1), against q0 (the product settings, experiments build); C4 and C3,
# alternated, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_q}
mkdir -p $O
for k in 1 2 3; do
  for v in q0 q1; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/c4_${v}_$k.log 2>&1 || { tail -5 $O/c4_${v}_$k.log; exit 1; }
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 100000000 Imp3D gossip 200 > $O/c3_${v}_$k.log 2>&1 || { tail -5 $O/c3_${v}_$k.log; exit 1; }
    echo "$v $k: C4 $(grep -o '[0-9.]* ms/round kernel' $O/c4_${v}_$k.log | head -1) | C3 $(grep -o '[0-9.]* ms/round kernel' $O/c3_${v}_$k.log | head -1)"
  done
done
