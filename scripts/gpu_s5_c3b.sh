#!/bin/bash
# C3 after the tiled random-edge delivery pass (time, kernel trace, gossip parity), and the
# 512-thread tile variant of the headline kernel; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out/c3b
n=gossip_Imp3D_100000000
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3b/$n -o kt -- python3 tools/perf_round.py 100000000 Imp3D gossip 20 > gpurun_out/c3b/$n.log 2>&1 || { tail -20 gpurun_out/c3b/$n.log; exit 1; }
grep -v "^E2\|^W2" gpurun_out/c3b/$n.log | tail -1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_baseline_sizes.py tests/test_gpu_rccl.py -x -q --timeout 300 --timeout-method thread -k "gossip or c3 or golden or live or variant" > gpurun_out/pytest_c3.log 2>&1 || { tail -30 gpurun_out/pytest_c3.log; exit 1; }
tail -1 gpurun_out/pytest_c3.log
timeout -k 10 300 python -u tools/ablate.py run 1000000000 base,t512m6,base
