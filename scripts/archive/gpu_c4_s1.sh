#!/bin/bash
# C4 coarse-bin size sweep (experiments build, GP_FB_S1D = shift of s1): parity of the full push-sum
# tests at each shift, then ms/round at P = 1e8 on the same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/c4_s1}
mkdir -p $O
for d in ${DS:--1 1}; do
  GP_FB_S1D=$d timeout -k 10 300 python -u tools/c4_variant_check.py > $O/check_$d.log 2>&1 || { tail -30 $O/check_$d.log; exit 1; }
  echo "s1 shift $d parity: $(tail -1 $O/check_$d.log)"
done
for d in 0 ${DS:--1 1} 0; do
  GP_FB_S1D=$d GP_EXP=1 timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 40 > $O/perf_$d.log 2>&1 || { tail -5 $O/perf_$d.log; exit 1; }
  echo "s1 shift $d: $(grep -o 'preroll.*' $O/perf_$d.log | tail -1)"
done
