#!/bin/bash
# The tile kernel's priority settings at the other sizes: C2 (3D push-sum, n = 1e6, the 1024-thread
# build), line push-sum n = 1000 and 3D push-sum n = 1e8 -- the product against the same experiments
# build without them (-DGP_SETPRIO=0, build/ablate/lib_sp0.so), alternated.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_prio_small}
mkdir -p $O
for k in 1 2 3; do
  for v in prod sp0; do
    if [ $v = sp0 ]; then E="GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_sp0.so"; else E="GP_EXP=1"; fi
    env $E timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 400 > $O/c2_${v}_$k.log 2>&1 || { tail -5 $O/c2_${v}_$k.log; exit 1; }
    env $E timeout -k 10 200 python3 tools/perf_round.py 1000 line push-sum 400 > $O/l_${v}_$k.log 2>&1 || { tail -5 $O/l_${v}_$k.log; exit 1; }
    env $E timeout -k 10 200 python3 tools/perf_round.py 100000000 3D push-sum 60 > $O/g_${v}_$k.log 2>&1 || { tail -5 $O/g_${v}_$k.log; exit 1; }
    echo "$v $k: C2 $(grep -o 'wall [0-9.]* ms/round' $O/c2_${v}_$k.log | head -1) | line $(grep -o 'wall [0-9.]* ms/round' $O/l_${v}_$k.log | head -1) | 3D 1e8 $(grep -o '[0-9.]* ms/round kernel' $O/g_${v}_$k.log | head -1)"
  done
done
