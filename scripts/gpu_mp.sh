#!/bin/bash
# Multi-process rehearsal on one GPU: 2 ranks (one process each) pinned to device 0,
# RCCL inside the library; small lattice; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
GP_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus ${NP:-2} --steps 5 --warmup 1 --nodes ${NODES:-8000000} --no-cpu > gpurun_out/mp.json 2> gpurun_out/mp.err
rc=$?
tail -30 gpurun_out/mp.err; cat gpurun_out/mp.json
exit $rc
