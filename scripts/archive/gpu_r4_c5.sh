#!/bin/bash
# The P = 1e9 parity segments (activation, steady state, alert peak, tail, determinism).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c5}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=10 \
  tests/test_gpu_parity.py -k "full_size_1e9" > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; exit $rc
