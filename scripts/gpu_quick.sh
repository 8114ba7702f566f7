#!/bin/bash
# Parity tests + steady-state round timing for the main configs; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/perf.log 2>&1 &&
timeout -k 10 300 python -u tools/perf_round.py 1000000 3D push-sum 200 >> gpurun_out/perf.log 2>&1 &&
timeout -k 10 300 python -u tools/perf_round.py 100000000 Imp3D gossip 20 >> gpurun_out/perf.log 2>&1 &&
timeout -k 10 300 python -u tools/perf_round.py 100000000 full push-sum 5 >> gpurun_out/perf.log 2>&1
