#!/bin/bash
# Round-2 end state on the product library: smoke(), the GPU test suite, the headline
# bench (HBM-traffic passes inside) + its rocprofv3 kernel trace, kernel traces of the
# other BASELINE configurations, and the C5 workload run to convergence.
export TMPDIR=/tmp
O=${O:-gpurun_out/final2}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
python3 tools/kt_steady.py $O/prof_kt k_ps_tile --last 20
for cfg in "1000000 3D push-sum 300" "100000000 Imp3D gossip 20" "100000000 full push-sum 10"; do
  set -- $cfg; d=$O/cfg_$3_$2_$1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o kt -- python3 tools/perf_round.py $cfg > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  grep -v "^E2\|^W2" $d.log | tail -2
  python3 tools/kt_steady.py $d k_ --last 10
done
timeout -k 10 600 python -u tools/converge.py 1000000000 Imp3D push-sum 1 $O/c5_converge_1e9.json 2> $O/converge.err
rc=$?; tail -3 $O/converge.err; exit $rc
