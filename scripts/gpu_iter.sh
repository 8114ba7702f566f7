#!/bin/bash
# Iteration check: push-sum parity subset, then per-node counters and time/HBM bytes (Imp3D, 3D at 1e9); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread -k "${PTK:-push or golden or live or close}" > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
VARIANTS="${PV:-GP_EXP=1}" bash scripts/gpu_pmcprobe.sh || exit 1
VARIANTS="${PV:-GP_EXP=1}" bash scripts/gpu_probe.sh || exit 1
TOPO=3D VARIANTS="${PV:-GP_EXP=1}" bash scripts/gpu_probe.sh
