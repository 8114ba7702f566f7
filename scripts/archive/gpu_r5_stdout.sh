#!/bin/bash
# bench.py's stdout holds only the JSON line at N > 1 (gloo's connection messages moved to stderr):
# the launcher tests, torch.distributed.run with two ranks on one GPU, and bench.py --gpus 2 at
# 10^9 nodes (region rounds: the roofline's kernel time is the sum of the region launches).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_stdout}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_launcher.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GP_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --nodes 8000000 --no-cpu > $O/torchrun.out 2> $O/torchrun.err || { tail -20 $O/torchrun.err; exit 1; }
echo "torchrun stdout lines: $(grep -c '' $O/torchrun.out)"; head -c 300 $O/torchrun.out; echo
GP_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-traffic > $O/bench_w2.out 2> $O/bench_w2.err || { tail -20 $O/bench_w2.err; exit 1; }
echo "bench --gpus 2 stdout lines: $(grep -c '' $O/bench_w2.out)"
python3 -c "
import json; d=json.loads(open('$O/bench_w2.out').read()); r=d['roofline']
print('rehearsal W=2 1e9: %.1f ms/round, kernel %.3f ms/round (%s)' % (d['ms_per_step'], r['kernel_avg_ms'], r['kernel']))"
