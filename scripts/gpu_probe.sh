#!/bin/bash
# Round time + HBM bytes per node-round for variants (tools/traffic_probe.py); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/traffic_probe.py ${N:-1000000000} ${TOPO:-Imp3D} ${ALG:-push-sum} ${KSUB:-k_ps_tile} ${VARIANTS:-default} || exit 1
