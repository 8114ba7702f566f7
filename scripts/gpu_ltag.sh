#!/bin/bash
# Edge-tag in-edge pass (opt-in GP_LTAG=1): tile-kernel parity (tags on / off), then A/B of the
# steady-state round at P = 1e9 (GP_LTAG=0 = Philox redraw, the default); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ltag.log 2>&1 || { tail -30 gpurun_out/pytest_ltag.log; exit 1; }
tail -2 gpurun_out/pytest_ltag.log
: > gpurun_out/ab_ltag.log
for i in 1 2; do
  for v in 0 1; do
    echo "== GP_LTAG=$v $(GP_LTAG=$v timeout -k 10 200 python -u tools/perf_round.py 1000000000 Imp3D push-sum 10 | grep -o 'k_ps_tile<[A-Z0-9]*>: [0-9.]* ms')" >> gpurun_out/ab_ltag.log || exit 1
  done
done
cat gpurun_out/ab_ltag.log
