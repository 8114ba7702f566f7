#!/bin/bash
# Own-line L2 touch A/B (time + HBM bytes), phase stamps; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_notouch.so" bash scripts/gpu_probe.sh || exit 1
timeout -k 10 300 python -u tools/ablate.py run 1000000000 base,notouch,stamps,base || exit 1
