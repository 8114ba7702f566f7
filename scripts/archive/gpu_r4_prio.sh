#!/bin/bash
# Headline kernel: wave priority raised while a node slot issues its loads (prio1) and also while the
# in-edge pass issues its gathers (prio2), against the same build without (base); tools/ablate.py
# variants, alternated, same box, P = 1e9.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_prio}
mkdir -p $O
for k in 1 2; do
  for v in base prio1 prio2; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 30 > $O/perf_${v}_$k.log 2>&1 || { tail -5 $O/perf_${v}_$k.log; exit 1; }
    echo "$v $k: $(grep -o '[0-9.]* ms/round kernel' $O/perf_${v}_$k.log | head -1)"
  done
done
