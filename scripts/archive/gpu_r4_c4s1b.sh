#!/bin/bash
# C4 fused: coarse-bin size 0 / -1 / -2 below the rule, alternated three times, 80 rounds each (same box).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4s1b}
mkdir -p $O
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o 'kernel [0-9.]* ms/round' $O/perf_$l.log | head -1) $(grep -o 'wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2 3; do
  run d0_$k GP_EXP=1 && run m1_$k GP_EXP=1 GP_FB_S1D=-1 && run m2_$k GP_EXP=1 GP_FB_S1D=-2 || exit 1
done
