#!/bin/bash
# Headline kernel: the next tile's in-edge senders LDS-DMA'd during this tile's node phase
# (build/ablate/lib_sndpf.so, -DGP_SND_PF=1; SLOTS 1216 -> 1152 for the buffer) against loading them at
# the tile's start (the product), C5 P = 1e9, same box, alternated; variant parity first.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_sndpf}; mkdir -p $O
V=build/ablate/lib_sndpf.so
for c in "512000 Imp3D push-sum 300" "8000000 Imp3D push-sum 150"; do
  GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 timeout -k 10 300 python3 tools/variant_parity.py $c > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
  tail -1 $O/parity.log
done
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o '[0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2 3; do
  run p$k GP_X=0 && run sndpf$k GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 || exit 1
done
