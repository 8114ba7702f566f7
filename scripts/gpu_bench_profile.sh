#!/bin/bash
# Headline bench + rocprofv3 kernel-trace/stats of the same command + separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) over the timed rounds; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --no-cpu --steps 20 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_kt.json 2> gpurun_out/bench_kt.err &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o f -- python3 bench.py --no-cpu --steps 10 --warmup 0 ${BENCH_ARGS} > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o w -- python3 bench.py --no-cpu --steps 10 --warmup 0 ${BENCH_ARGS} > gpurun_out/bench_w.json 2> gpurun_out/bench_w.err
