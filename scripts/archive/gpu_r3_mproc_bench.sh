#!/bin/bash
# bench.py as the driver launches it for N > 1 (torch.distributed.run, one process per rank), at the
# BASELINE size, with every rank pinned to the one GPU (GP_BENCH_DEVICE=0: RCCL socket transport on
# loopback, see bench.py) -- a rehearsal of the multi-GPU code path; its timing is not a multi-GPU number.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_mproc}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl_multiproc.py -x -v --timeout 200 --timeout-method thread --durations=10 > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
echo "parity: $(tail -1 $O/pytest.log)"
for W in ${WS:-2 4}; do
  GP_BENCH_DEVICE=0 timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
    --master-addr 127.0.0.1 --master-port 2954$W bench.py --gpus $W --steps 10 --warmup 2 \
    > $O/bench_c5_w$W.json 2> $O/bench_c5_w$W.err || { tail -40 $O/bench_c5_w$W.err; exit 1; }
  cat $O/bench_c5_w$W.json
done
