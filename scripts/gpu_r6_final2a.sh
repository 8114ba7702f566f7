#!/bin/bash
# Round-6 end state (after the wait / flat-store changes), part A: smoke and the whole GPU suite.
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_final3}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=40 > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -2; grep FAILED $O/pytest_gpu.log | head; exit $rc
