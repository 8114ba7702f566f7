#!/bin/bash
# Round-6 end state on one MI355X: smoke, the whole GPU suite (BASELINE-size rank-process runs
# included), C2 to convergence on the product kernel, bench (traffic + CPU baseline), kernel trace.
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_final}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=40 > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -2; grep FAILED $O/pytest_gpu.log | head; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 tools/converge.py 1000000 3D push-sum 1 $O/c2_converge.json > $O/c2_converge.log 2>&1 || { tail -5 $O/c2_converge.log; exit 1; }
tail -2 $O/c2_converge.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
python3 tools/kt_steady.py $O/prof_kt k_ps_tile --last 20
rm -f $O/prof_kt/*/kt_kernel_trace.csv $O/prof_kt/kt_kernel_trace.csv 2>/dev/null; true
