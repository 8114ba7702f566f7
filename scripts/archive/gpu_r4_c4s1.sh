#!/bin/bash
# C4 fused: coarse-bin size sweep below the rule (GP_FB_S1D, experiments build), same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4s1}
mkdir -p $O
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 40 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o 'wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
run d0 GP_EXP=1 && run m1 GP_EXP=1 GP_FB_S1D=-1 && run m2 GP_EXP=1 GP_FB_S1D=-2 && run m3 GP_EXP=1 GP_FB_S1D=-3 || exit 1
run d0b GP_EXP=1 && run m1b GP_EXP=1 GP_FB_S1D=-1 && run m2b GP_EXP=1 GP_FB_S1D=-2 && run m3b GP_EXP=1 GP_FB_S1D=-3 || exit 1
for d in -1 -2 -3; do
  GP_EXP=1 GP_FB_S1D=$d timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt$d -o kt -- python3 tools/perf_round.py 100000000 full push-sum 20 > $O/kt$d.log 2>&1 || { tail -5 $O/kt$d.log; exit 1; }
  echo "S1D=$d"; python3 tools/kt_steady.py $O/kt$d k_fb_ --last 20 || true
done
