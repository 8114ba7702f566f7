#!/bin/bash
# C5 (10^9-node Imp3D push-sum) run to convergence with the final code.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_conv}
mkdir -p $O
timeout -k 10 200 python -u tools/converge.py 1000000000 Imp3D push-sum 1 $O/c5_converge_1e9.json > $O/converge.log 2>&1 || { tail -20 $O/converge.log; exit 1; }
tail -1 $O/converge.log
