#!/bin/bash
# C5 at W = 8 virtual ranks: HBM bytes and SQ counters per dispatch of the REMOTE round kernel for two
# libraries (tools/pack_probe.py: each counter pass its own rocprofv3 run).  VARIANTS, O.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_remote_pmc}; mkdir -p $O
for v in $VARIANTS; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 600 python3 -u tools/pack_probe.py 1000000000 Imp3D push-sum 8 "k_ps_tile<3, true>" > $O/probe_$v.log 2>&1 || { tail -20 $O/probe_$v.log; exit 1; }
  echo "== $v"; cat $O/probe_$v.log
done
