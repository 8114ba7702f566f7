#!/bin/bash
# HBM traffic per pass (request-size counters) of C3 (push-form gossip column kernel) and C4
# (full push-sum send / split / fold), and the C4 kernel trace.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_traffic}
mkdir -p $O
timeout -k 10 400 python3 tools/traffic_probe.py 100000000 Imp3D gossip k_gossip_col > $O/c3.txt 2>&1 || { tail -5 $O/c3.txt; exit 1; }
cat $O/c3.txt
for k in k_fb_send k_fb_split k_fb_fold; do
  timeout -k 10 400 python3 tools/traffic_probe.py 100000000 full push-sum $k > $O/c4_$k.txt 2>&1 || { tail -5 $O/c4_$k.txt; exit 1; }
  echo "$k $(cat $O/c4_$k.txt)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c4_kt -o kt -- python3 tools/perf_round.py 100000000 full push-sum 20 > $O/c4_kt.log 2>&1 || { tail -5 $O/c4_kt.log; exit 1; }
python3 tools/kt_steady.py $O/c4_kt k_fb --last 20
