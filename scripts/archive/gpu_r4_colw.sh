#!/bin/bash
# C3 column kernel with wave priority at 4 / 5 (product) / 6 waves per SIMD (-DGP_COL_WAVES, experiments
# builds; 6 spills 76 B), alternated, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_colw}
mkdir -p $O
for k in 1 2 3; do
  for v in cw5 cw4 cw6; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 100000000 Imp3D gossip 200 > $O/c3_${v}_$k.log 2>&1 || { tail -5 $O/c3_${v}_$k.log; exit 1; }
    echo "$v $k: $(grep -o '[0-9.]* ms/round kernel' $O/c3_${v}_$k.log | head -1)"
  done
done
