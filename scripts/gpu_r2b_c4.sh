#!/bin/bash
# C4 full push-sum: round time and HBM bytes per node-round of each binning kernel; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in k_fb_send k_fb_split k_fb_fold; do
  echo "== $k"; N=100000000 TOPO=full ALG=push-sum KSUB=$k VARIANTS="default" bash scripts/gpu_probe.sh || exit 1
done
