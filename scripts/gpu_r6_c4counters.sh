#!/bin/bash
# C4 on one GPU (full push-sum, P = 1e8): per-pass HBM bytes (request-size counters), SQ
# instruction / cycle counters, and a kernel trace of the split and the fused fold.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_c4cnt}; mkdir -p $O
for k in k_fb_split k_fb_fold; do
  timeout -k 10 500 python3 tools/traffic_probe.py 100000000 full push-sum $k default > $O/${k}_traffic.txt 2>&1 || { tail $O/${k}_traffic.txt; exit 1; }
  cat $O/${k}_traffic.txt
  timeout -k 10 500 python3 tools/pmc_probe.py 100000000 full push-sum $k default > $O/${k}_pmc.txt 2>&1 || { tail $O/${k}_pmc.txt; exit 1; }
  cat $O/${k}_pmc.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/perf_round.py 100000000 full push-sum 40 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
python3 tools/kt_steady.py $O/kt k_fb_split --last 40 && python3 tools/kt_steady.py $O/kt k_fb_fold --last 40
rm -f $O/kt/*/kt_kernel_trace.csv $O/kt/kt_kernel_trace.csv 2>/dev/null; true
