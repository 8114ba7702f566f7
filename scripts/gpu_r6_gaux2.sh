#!/bin/bash
# C5 one GPU, alternated same-box timing: the product's gathers (nt) vs sc0 nt on the in-edge
# gathers (lib_gaux3) vs sc0 nt on every single-use staging copy too (lib_gall3), vs sc0 sc1.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_gaux2}; mkdir -p $O
run() { local l=$1; shift; env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 30 > $O/$l.log 2>&1 || { tail -5 $O/$l.log; return 1; }; echo "$l: $(grep -o '[0-9.]* ms/round kernel' $O/$l.log | head -1)"; }
for i in 1 2 3; do
  run base_$i GP_EXP=1 && run aux3_$i GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gaux3.so && run all3_$i GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gall3.so && run aux17_$i GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gaux17.so || exit 1
done
