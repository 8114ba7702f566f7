#!/bin/bash
# Round-6 end state, part B: bench (traffic passes + CPU baseline), its kernel trace, C2 and C5 to
# convergence.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_final3}
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
python3 tools/kt_steady.py $O/prof_kt k_ps_tile --last 20
rm -f $O/prof_kt/*/kt_kernel_trace.csv $O/prof_kt/kt_kernel_trace.csv 2>/dev/null
timeout -k 10 300 python3 tools/converge.py 1000000 3D push-sum 1 $O/c2_converge.json > $O/c2_converge.log 2>&1 || { tail -5 $O/c2_converge.log; exit 1; }
tail -1 $O/c2_converge.log
timeout -k 10 300 python3 tools/converge.py 1000000000 Imp3D push-sum 1 $O/c5_converge_1e9.json > $O/c5_converge.log 2>&1 || { tail -5 $O/c5_converge.log; exit 1; }
tail -1 $O/c5_converge.log
