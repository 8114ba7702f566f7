#!/bin/bash
# Round-4 state, part 1: smoke() and the whole GPU suite (incl. the P = 1e9 alert-phase sampled-oracle
# checks, the recorded 1e8 oracle runs, the launchers).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_state}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=60 > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -3; grep FAILED $O/pytest_gpu.log | head; exit $rc
