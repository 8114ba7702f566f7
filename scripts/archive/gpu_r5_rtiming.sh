#!/bin/bash
# Kernel timing of region rounds (events around each region launch): multi-rank parity and
# launcher tests, then bench.py --gpus 2 at 10^9 nodes with both ranks on one GPU (a rehearsal,
# socket transport) to see the roofline's kernel time per round.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_rtiming}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py tests/test_gpu_rccl_multiproc.py tests/test_gpu_launcher.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GP_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-traffic > $O/bench_w2.json 2> $O/bench_w2.err || { tail -20 $O/bench_w2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_w2.json')); r=d['roofline']
print('rehearsal W=2: %.1f ms/round, kernel %.3f ms/round (%s), achieved %.0f GB/s' % (d['ms_per_step'], r['kernel_avg_ms'], r['kernel'], r['achieved']))"
