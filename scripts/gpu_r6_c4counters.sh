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
# the W = 8 model again (the state of the commit)
d=$O/vr_c4w8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 100000000 full push-sum 8 20 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python3 tools/mgpu_model.py model $d 100000000 full push-sum 8 20 $O/model_c4w8.json > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('$O/model_c4w8.json'))
print('c4w8: rank compute max %.3f ms, regions %s, sched %.3f (128) / %.3f (64) ms' % (max(d['rank_compute_ms']), d['full_fused_regions'], d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled']))
print('   per-slab kernels', {k: round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()})"
rm -f $d/*/kt_kernel_trace.csv $d/kt_kernel_trace.csv 2>/dev/null; true
