#!/bin/bash
# Round timing of the main configs with the current build, then the whole GPU
# test suite; run via gpurun.  PYTEST_ARGS narrows the tests.
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/perf.log
for cfg in "1000000000 Imp3D push-sum 10" "1000000 3D push-sum 300" "100000000 Imp3D gossip 20" ${EXTRA_PERF}; do
  timeout -k 10 300 python -u tools/perf_round.py $cfg >> gpurun_out/perf.log 2>&1 || { cat gpurun_out/perf.log; exit 1; }
done
cat gpurun_out/perf.log
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
exit $rc
