#!/bin/bash
# Session-5 checkpoint: smoke, full GPU suite, headline bench + kernel trace, and the C5
# run to convergence (with its activation / steady round times); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_round.sh || exit 1
timeout -k 10 900 python -u tools/converge.py 1000000000 Imp3D push-sum 1 gpurun_out/converge.json 2> gpurun_out/converge.err
rc=$?
tail -3 gpurun_out/converge.err
exit $rc
