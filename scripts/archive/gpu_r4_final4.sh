#!/bin/bash
# Round-4 end state after the fold-grid change: smoke, GPU suite, bench (traffic + CPU baseline), kernel
# trace, C4 ms/round, and the W = 8 virtual-rank models of C5 and C4.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_final4}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=30 > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -2; grep FAILED $O/pytest_gpu.log | head; [ $rc = 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
python3 tools/kt_steady.py $O/prof_kt k_ps_tile --last 20
for k in 1 2; do
  timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/c4_$k.log 2>&1 || { tail -5 $O/c4_$k.log; exit 1; }
  tail -1 $O/c4_$k.log
done
for cfg in "1000000000 Imp3D push-sum c5" "100000000 full push-sum c4"; do
  set -- $cfg; d=$O/vr_$4_w8
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $1 $2 $3 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python3 tools/mgpu_model.py model $d $1 $2 $3 8 10 $O/model_$4_w8.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/model_$4_w8.json')); print('$4 W=8', {k:round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'], [(m['link_gbps'], round(m['round_ms_as_scheduled'],3), '%.3g' % m['node_updates_per_s_overlapped']) for m in d['model']])"
done
