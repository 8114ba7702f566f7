#!/bin/bash
# Parity tests (default kernel) + steady-state A/B of the round-kernel variants; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
for v in wave tile; do
  GP_KERNEL=$v timeout -k 10 300 python -u tools/perf_round.py ${N:-1000000000} Imp3D push-sum 10 >> gpurun_out/perf_ab.log 2>&1 || exit 1
  GP_KERNEL=$v timeout -k 10 300 python -u tools/perf_round.py 100000000 Imp3D gossip 20 >> gpurun_out/perf_ab.log 2>&1 || exit 1
  GP_KERNEL=$v timeout -k 10 300 python -u tools/perf_round.py 1000000 3D push-sum 200 >> gpurun_out/perf_ab.log 2>&1 || exit 1
done
