#!/bin/bash
# C5 one GPU: cache-policy bits of the in-edge (s, w) gathers of k_ps_tile (LDS-DMA, 16 B per used
# in-edge): HBM request sizes and round time per variant (build/ablate/lib_gaux<bits>.so, built from
# patched copies; the product uses nt = 2).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_gaux}; mkdir -p $O
timeout -k 10 900 python3 tools/traffic_probe.py 1000000000 Imp3D push-sum k_ps_tile GP_EXP=1 \
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gaux0.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gaux17.so \
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gaux3.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gaux16.so \
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_gaux1.so GP_EXP=1 > $O/traffic.txt 2>&1 || { tail $O/traffic.txt; exit 1; }
cat $O/traffic.txt
