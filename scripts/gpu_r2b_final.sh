#!/bin/bash
# Round-2 checkpoint on the product library: smoke(), the GPU test suite, the headline
# bench (HBM-traffic passes inside) and a rocprofv3 kernel trace of the same command.
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 900 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
cat gpurun_out/final/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 > gpurun_out/final/bench_kt.json 2> gpurun_out/final/bench_kt.err || { tail -20 gpurun_out/final/bench_kt.err; exit 1; }
cat gpurun_out/final/bench_kt.json
python3 tools/kt_steady.py gpurun_out/final/prof_kt k_ps_tile --last 20
