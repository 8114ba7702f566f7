#!/bin/bash
# Multi-process RCCL rehearsal on one GPU: per-rank NCCL_HOSTID (socket transport on loopback).
# 1) rank processes vs a single-process run, bit-exact; 2) bench.py under torch.distributed.run, 2 ranks.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_mproc}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rccl_multiproc.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
echo "parity: $(tail -1 $O/pytest.log)"
GP_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${NPROC:-2} --steps ${STEPS:-10} --warmup 2 \
  --nodes ${NODES:-8000000} > $O/bench_w${NPROC:-2}.json 2> $O/bench_w${NPROC:-2}.err || { tail -40 $O/bench_w${NPROC:-2}.err; exit 1; }
cat $O/bench_w${NPROC:-2}.json
if [ -n "$FULL" ]; then
  GP_MPROC_FULL=1 timeout -k 10 1000 python -u -m pytest tests/test_gpu_rccl_multiproc.py -k baseline_size -x -v --timeout 950 --timeout-method thread > $O/pytest_baseline_sizes.log 2>&1 || { tail -60 $O/pytest_baseline_sizes.log; exit 1; }
  echo "baseline sizes: $(tail -1 $O/pytest_baseline_sizes.log)"
fi
