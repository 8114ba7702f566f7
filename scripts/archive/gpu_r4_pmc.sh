#!/bin/bash
# SQ counters of the headline kernel, the product against the round-3 scheduling (no wave priority, no
# stealing, 8-plane windows: tools/ablate.py sched0 + GP_WX=8), P = 1e9 (tools/pmc_probe.py).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_pmc}
mkdir -p $O
timeout -k 10 900 python3 tools/pmc_probe.py 1000000000 Imp3D push-sum "k_ps_tile<3" default "GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_sched0.so,GP_EXP=1,GP_WX=8" > $O/pmc.txt 2>&1 || { tail -20 $O/pmc.txt; exit 1; }
cat $O/pmc.txt
