#!/bin/bash
# Round-close parity + counter list; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "round_close or golden" > gpurun_out/pytest_close.log 2>&1 || { tail -30 gpurun_out/pytest_close.log; exit 1; }
tail -2 gpurun_out/pytest_close.log
