#!/bin/bash
# C4 split pass: XCD-grouped work items (build/ablate/lib_xcdmap.so, -DGP_FB_XCDMAP=1) against the
# product -- parity (oracle + product at 1e8), split-pass HBM bytes, ms/round at P = 1e8 (same box).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4}
mkdir -p $O
V=build/ablate/lib_xcdmap.so
GOSSIP_HIP_LIB_EXPERIMENT=$V timeout -k 10 400 python3 -u tools/c4_variant_check.py > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
tail -2 $O/check.log
timeout -k 10 600 python3 tools/traffic_probe.py 100000000 full push-sum k_fb_split default "GOSSIP_HIP_LIB_EXPERIMENT=$V,GP_EXP=1" > $O/split_traffic.txt 2>&1 || { tail -5 $O/split_traffic.txt; exit 1; }
cat $O/split_traffic.txt
for v in p x p x; do
  if [ $v = x ]; then export GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1; else unset GOSSIP_HIP_LIB_EXPERIMENT GP_EXP; fi
  timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 40 > $O/perf_$v.log 2>&1 || { tail -5 $O/perf_$v.log; exit 1; }
  echo "$v: $(grep -o 'wall [0-9.]* ms/round' $O/perf_$v.log | head -1)"
done
