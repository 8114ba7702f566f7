#!/bin/bash
# bench.py default run with the CPU baseline on the benchmarked workload (P = 1e9).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_bench_cpu}
mkdir -p $O
t0=$(date +%s)
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
echo "bench.py wall $(( $(date +%s) - t0 )) s" | tee -a $O/bench.err
cat $O/bench.json; tail -8 $O/bench.err
