#!/bin/bash
# walk 3: x-window width variants (time + HBM bytes) and phase stamps; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
VARIANTS="GP_EXP=1,GP_WX=4 GP_EXP=1,GP_WX=16 GP_EXP=1,GP_WX=32 GP_EXP=1,GP_WX=125" bash scripts/gpu_probe.sh || exit 1
timeout -k 10 300 python -u tools/ablate.py run 1000000000 base,stamps
