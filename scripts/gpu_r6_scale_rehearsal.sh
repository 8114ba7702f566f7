#!/bin/bash
# The driver's N>1 bench command, rehearsed on a one-GPU box: two ranks on device 0
# (GP_BENCH_DEVICE, RCCL socket transport) through torch.distributed.run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_scale; mkdir -p $O
GP_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_w2.json 2> $O/bench_w2.err || { tail -30 $O/bench_w2.err; exit 1; }
cat $O/bench_w2.json
