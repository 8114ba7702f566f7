#!/bin/bash
# Round check: smoke(), full GPU test suite, then the headline bench + rocprofv3
# kernel-trace and PMC passes (scripts/gpu_bench_profile.sh); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
bash scripts/gpu_bench_profile.sh || exit 1
cat gpurun_out/bench.json
