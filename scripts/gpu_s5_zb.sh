#!/bin/bash
# Wave-end j+-1 neighbours staged in LDS (no fallback gathers): push-sum parity, then
# A/B against the previous build; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "push or golden or live or variant or c5" > gpurun_out/pytest_zb.log 2>&1 || { tail -30 gpurun_out/pytest_zb.log; exit 1; }
tail -1 gpurun_out/pytest_zb.log
timeout -k 10 400 python -u tools/ablate.py run 1000000000 head,base,head,base || exit 1
