#!/bin/bash
# Per-node instruction counters (tools/pmc_probe.py) for variants; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/pmc_probe.py ${N:-1000000000} ${TOPO:-Imp3D} ${ALG:-push-sum} ${KSUB:-k_ps_tile} ${VARIANTS:-default} 2>&1 | tee gpurun_out/pmcprobe.log
