#!/bin/bash
# Headline kernel at 6 waves per SIMD (build/ablate/lib_w6.so: -DGP_MINB=6 -DGP_HMAX=1000 -- 80 VGPRs with
# 11 spilled, 26 976 B of LDS) against the product (5 waves, 96 VGPRs), C5 P = 1e9, same box, alternated.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_w6}; mkdir -p $O
V=build/ablate/lib_w6.so
timeout -k 10 300 env GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 python3 tools/variant_parity.py 512000 Imp3D push-sum 120 > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o '[0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2; do
  run p$k GP_X=0 && run w6_$k GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 || exit 1
done
