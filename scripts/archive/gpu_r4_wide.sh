#!/bin/bash
# Tiled-kernel size classes: 256 threads x 4 nodes (GP_WIDE=0) vs 1024 x 1 (GP_WIDE=1, gp_round_wide.hip),
# wall per round at small and medium populations (same box), then the product's own choice.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_wide}
mkdir -p $O
for cfg in "1000000 3D push-sum 2000" "1000000 Imp3D push-sum 2000" "8000000 3D push-sum 400" "8000000 Imp3D push-sum 400" "27000000 Imp3D push-sum 200" "1000 line push-sum 4000" "1000000 3D gossip 400"; do
  set -- $cfg
  for w in 0 1; do
    GP_EXP=1 GP_WIDE=$w timeout -k 10 200 python3 tools/perf_round.py $1 $2 $3 $4 > $O/perf_$2_$3_$1_w$w.log 2>&1 || { tail -5 $O/perf_$2_$3_$1_w$w.log; exit 1; }
    echo "$2 $3 n=$1 wide=$w: $(grep -o 'k_[a-z_+<>A-Z0-9:]*: [0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$2_$3_$1_w$w.log) $(grep -o 'no events: wall [0-9.]* ms/round' $O/perf_$2_$3_$1_w$w.log)"
  done
done
