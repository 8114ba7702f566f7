#!/bin/bash
# Round 5 start: default bench (CPU baseline now on every scheduler core) + the
# un-gated C5 two-process RCCL case.
set -o pipefail
O=gpurun_out/r5_start; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
nproc > $O/nproc.txt; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/nproc.txt
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.json
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_rccl_multiproc.py -k "baseline_size" > $O/mproc.log 2>&1 || { tail -20 $O/mproc.log; exit 1; }
tail -3 $O/mproc.log
