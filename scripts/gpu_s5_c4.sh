#!/bin/bash
# Full-topology push-sum (C4): parity (golden/live/C4 at 1e8 to convergence), then the
# steady-state round with a kernel trace; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "full or golden or c4" > gpurun_out/pytest_c4.log 2>&1 || { tail -30 gpurun_out/pytest_c4.log; exit 1; }
tail -2 gpurun_out/pytest_c4.log
n=push-sum_full_100000000
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4/$n -o kt -- python3 tools/perf_round.py 100000000 full push-sum 10 > gpurun_out/c4/$n.log 2>&1 || { tail -20 gpurun_out/c4/$n.log; exit 1; }
grep -v "^E2\|^W2" gpurun_out/c4/$n.log | tail -2
