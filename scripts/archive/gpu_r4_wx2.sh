#!/bin/bash
# Headline kernel with wave priority and work stealing: walk-3 x-window of 16 (product) / 24 / 32 / 48 / 64 planes
# (GP_WX, experiments build), alternated, same box, P = 1e9.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_wx2}
mkdir -p $O
for k in 1 2; do
  for w in 16 24 32 48 64; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so GP_WX=$w timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 40 > $O/perf_${w}_$k.log 2>&1 || { tail -5 $O/perf_${w}_$k.log; exit 1; }
    echo "wx=$w $k: $(grep -o '[0-9.]* ms/round kernel' $O/perf_${w}_$k.log | head -1)"
  done
done
