#!/bin/bash
# Iteration loop: tile-kernel parity + steady-state timing of the headline config; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
timeout -k 10 200 python -u tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/perf_iter.log 2>&1 || exit 1
GP_KERNEL=tile timeout -k 10 200 python -u tools/perf_round.py 100000000 Imp3D gossip 20 >> gpurun_out/perf_iter.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/perf_round.py 1000000 3D push-sum 200 >> gpurun_out/perf_iter.log 2>&1 || exit 1
cat gpurun_out/perf_iter.log
GP_EDGES=1 timeout -k 10 200 python -u tools/perf_round.py 1000000000 Imp3D push-sum 10 >> gpurun_out/perf_iter.log 2>&1 || exit 1
tail -1 gpurun_out/perf_iter.log
