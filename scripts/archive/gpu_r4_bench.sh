#!/bin/bash
# Round-4 state, part 2: the headline bench (HBM-traffic passes inside), its rocprofv3 kernel trace, and the
# two-rank rehearsal of bench.py --gpus 2 at the headline size (one GPU, RCCL sockets).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_state}
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o kt -- python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 2 > $O/bench_kt.json 2> $O/bench_kt.err || { tail -20 $O/bench_kt.err; exit 1; }
python3 tools/kt_steady.py $O/prof_kt k_ps_tile --last 20
GP_BENCH_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus 2 --steps 10 > $O/bench_gpus2_rehearsal.json 2> $O/bench_gpus2_rehearsal.err || { tail -20 $O/bench_gpus2_rehearsal.err; exit 1; }
cat $O/bench_gpus2_rehearsal.json
timeout -k 10 200 python -u tools/converge.py 1000000000 Imp3D push-sum 1 $O/c5_converge_1e9.json > $O/converge.log 2>&1 || { tail -20 $O/converge.log; exit 1; }
tail -1 $O/converge.log
