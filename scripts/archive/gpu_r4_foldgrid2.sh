#!/bin/bash
# C4 fused fold grid, fewer blocks: 2048 / 1024 / 512 / 256 (one per CU), experiments build (GP_FOLD_BLOCKS), alternated, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_foldgrid2}
mkdir -p $O
for k in 1 2 3; do
  for b in 2048 1024 512 256; do
    GP_EXP=1 GP_FOLD_BLOCKS=$b timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/c4_${b}_$k.log 2>&1 || { tail -5 $O/c4_${b}_$k.log; exit 1; }
    echo "blocks=$b $k: $(grep -o '[0-9.]* ms/round kernel' $O/c4_${b}_$k.log | head -1)"
  done
done
