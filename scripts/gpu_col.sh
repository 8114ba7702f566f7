#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "kernel_variant" > gpurun_out/pytest_kv.log 2>&1 &&
VARIANTS="GP_KERNEL=col GP_KERNEL=tile" bash scripts/gpu_perf.sh &&
VARIANTS="GP_KERNEL=col GP_KERNEL=tile" N=100000000 ALG=gossip R=20 bash scripts/gpu_perf.sh
