#!/bin/bash
# Multi-rank parity after the exchange-kernel priority change: virtual ranks, RCCL rank processes, launchers.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_mr}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl_multiproc.py tests/test_gpu_launcher.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
