#!/bin/bash
# Headline round timing of the current build, then the whole GPU test suite; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/perf.log 2>&1 || { cat gpurun_out/perf.log; exit 1; }
cat gpurun_out/perf.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
exit $rc
