#!/bin/bash
# Headline bench (its HBM-traffic passes run inside bench.py) + rocprofv3
# kernel-trace/stats of the same command; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_kt.json 2> gpurun_out/bench_kt.err
