#!/bin/bash
# Round-4 state on the product library: smoke(), the GPU test suite (incl. the P = 1e9
# alert-phase sampled-oracle checks and the recorded 1e8 runs), the headline bench (HBM-traffic passes inside) and
# its rocprofv3 kernel trace.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_state}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -20 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
python3 tools/kt_steady.py $O/prof_kt k_ps_tile --last 20
