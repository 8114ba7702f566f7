#!/bin/bash
# The sender prefetch as the product (GP_SND_PF=1) against the round-4 form (build/ablate/lib_snd0.so,
# -DGP_SND_PF=0), C5 P = 1e9, same box, alternated -- a second box for the record.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_sndpf2}; mkdir -p $O
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o '[0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2 3; do
  run sndpf$k GP_X=0 && run snd0_$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_snd0.so GP_EXP=1 || exit 1
done
