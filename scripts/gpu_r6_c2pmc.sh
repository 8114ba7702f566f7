#!/bin/bash
# C2: SQ instruction / cycle counters of k_ps_block (8-round launches), the product kernel and its
# no-node-work ablation (build/ablate/lib_c2nowork.so, built from a patched copy), then timing.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_c2pmc}; mkdir -p $O
timeout -k 10 400 python3 tools/pmc_probe.py 1000000 3D push-sum k_ps_block default GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_c2nowork.so,GP_KERNEL=block > $O/pmc.txt 2>&1 || { tail $O/pmc.txt; exit 1; }
cat $O/pmc.txt
timeout -k 10 200 env GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_c2nowork.so GP_KERNEL=block python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_nowork_abl.log 2>&1 && grep -o 'no events: wall [0-9.]* ms/round' $O/c2_nowork_abl.log
