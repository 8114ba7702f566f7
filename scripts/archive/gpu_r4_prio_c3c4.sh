#!/bin/bash
# s_setprio in the gossip column kernel (C3) and the full push-sum fold / split (C4): variant build with
# -DGP_COL_PRIO=1 -DGP_FB_PRIO=1 (build/ablate/lib_pall.so) against the same build without
# (lib_pnone.so), alternated, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_prio_c3c4}
mkdir -p $O
for k in 1 2 3; do
  for v in pnone pall; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 100000000 Imp3D gossip 200 > $O/c3_${v}_$k.log 2>&1 || { tail -5 $O/c3_${v}_$k.log; exit 1; }
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/c4_${v}_$k.log 2>&1 || { tail -5 $O/c4_${v}_$k.log; exit 1; }
    echo "$v $k: C3 $(grep -o '[0-9.]* ms/round kernel' $O/c3_${v}_$k.log | head -1) | C4 $(grep -o '[0-9.]* ms/round kernel' $O/c4_${v}_$k.log | head -1)"
  done
done
