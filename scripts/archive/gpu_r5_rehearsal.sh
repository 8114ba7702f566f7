#!/bin/bash
# bench.py on two and four rank processes at the headline size, all on one GPU (GP_BENCH_DEVICE=0: RCCL
# over sockets) -- the driver's --gpus N path with the round-5 exchange, and once under torch.distributed.run.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_rehearsal}; mkdir -p $O
GP_BENCH_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 --no-cpu --no-traffic > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { tail -20 $O/bench_gpus2.err; exit 1; }
cat $O/bench_gpus2.json
GP_BENCH_DEVICE=0 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 10 --warmup 2 --no-cpu --no-traffic > $O/bench_gpus4_torchrun.json 2> $O/bench_gpus4_torchrun.err || { tail -20 $O/bench_gpus4_torchrun.err; exit 1; }
cat $O/bench_gpus4_torchrun.json
