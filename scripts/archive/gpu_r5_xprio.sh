#!/bin/bash
# Rank processes sharing one GPU (socket transport): the exchange stream at the greatest priority
# against the default, with and without region rounds (experiments build, GP_XPRIO / GP_RREGIONS).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_xprio}; mkdir -p $O
run() {  # run <tag> <env...>
  local t=$1; shift
  env GP_EXP=1 "$@" timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_rccl_multiproc.py -k "4-64000 or 3-27000" --durations=5 > $O/$t.log 2>&1 || { tail -30 $O/$t.log; return 1; }
  echo "$t: $(grep -E 's call' $O/$t.log | tr -s ' ' | cut -c1-120 | paste -sd ';')"
}
run p1r1 GP_XPRIO=1 GP_RREGIONS=1 && run p0r1 GP_XPRIO=0 GP_RREGIONS=1 && run p1r0 GP_XPRIO=1 GP_RREGIONS=0 && run p0r0 GP_XPRIO=0 GP_RREGIONS=0
