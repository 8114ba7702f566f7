#!/bin/bash
# Per-phase cycle stamps of the push-sum tile kernel (experiments build with
# GP_STAMPS) and C3 column-march gossip: Imp3D vs 3D (cost of the in-edge path); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ablate.py run 1000000000 base,stamps || exit 1
for t in 3D Imp3D; do timeout -k 10 200 python -u tools/perf_round.py 100000000 $t gossip 20 || exit 1; done
