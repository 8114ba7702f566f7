#!/bin/bash
# Headline kernel: wave priority raised while the in-edge pass and each node slot issue their loads
# (prio2), and on through the staging copies (prio3), against base; three alternations, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_prio2}
mkdir -p $O
for k in 1 2 3; do
  for v in base prio2 prio3; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 40 > $O/perf_${v}_$k.log 2>&1 || { tail -5 $O/perf_${v}_$k.log; exit 1; }
    echo "$v $k: $(grep -o '[0-9.]* ms/round kernel' $O/perf_${v}_$k.log | head -1)"
  done
done
