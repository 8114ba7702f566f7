#!/bin/bash
# Push-sum column kernel: parity on the small variant cases and at 1e8, then a 1e9 timing probe.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_pscol}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "kernel_variant and col and push or large_imp3d_pushsum or test_golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_1e9.log 2>&1 || { tail -20 $O/perf_1e9.log; exit 1; }
grep -v "^W2\|^E2" $O/perf_1e9.log | tail -3
