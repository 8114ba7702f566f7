#!/bin/bash
# Headline kernel with wave priority: plain (temporal) loads / stores instead of non-temporal
# (tools/ablate.py plainld / plainst), x-windows of 4 / 16 planes (GP_WX, experiments build) against
# the product form; alternated, same box, P = 1e9.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_misc}
mkdir -p $O
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 40 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o '[0-9.]* ms/round kernel' $O/perf_$l.log | head -1)"
}
for k in 1 2; do
  run base$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so && run plainld$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_plainld.so && run plainst$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_plainst.so && run wx4_$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so GP_WX=4 && run wx16_$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so GP_WX=16 || exit 1
done
