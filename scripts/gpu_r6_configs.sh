#!/bin/bash
# Round-6 end state, every BASELINE config on one box with the final code: C1 through the CLI
# (line gossip, 1000 nodes, to convergence), C2 (block kernel, 4000 steady rounds), C3 (Imp3D gossip
# 1.005e8), C4 (full push-sum 1e8), C5 (Imp3D push-sum 1e9), steady-state kernel times.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_configs}; mkdir -p $O
timeout -k 10 120 gossipprotocol_amd/gossip 1000 line gossip > $O/c1_cli.log 2>&1 || { cat $O/c1_cli.log; exit 1; }
echo "C1: $(tail -1 $O/c1_cli.log)"
timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
echo "C2: $(head -1 $O/c2.log | cut -c1-250)"; grep "no events" $O/c2.log | head -1
timeout -k 10 200 python3 tools/perf_round.py 100000000 Imp3D gossip 200 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
echo "C3: $(head -1 $O/c3.log | cut -c1-250)"
timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 60 > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
echo "C4: $(head -1 $O/c4.log | cut -c1-250)"
timeout -k 10 240 python3 tools/perf_round.py 1000000000 Imp3D push-sum 60 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
echo "C5: $(head -1 $O/c5.log | cut -c1-250)"
