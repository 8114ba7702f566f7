#!/bin/bash
# Round-6 end state after the late C2 / C4 read changes: bench (traffic passes + CPU baseline), its
# kernel trace, C2 and C5 to convergence (scripts/gpu_r6_final2b.sh), and C4's modelled W = 8 round.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_final4}; mkdir -p $O
O=$O bash scripts/gpu_r6_final2b.sh || exit 1
d=$O/vr_c4w8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 100000000 full push-sum 8 20 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python3 tools/mgpu_model.py model $d 100000000 full push-sum 8 20 $O/model_c4w8.json > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('$O/model_c4w8.json'))
print('c4w8: rank compute max %.3f ms, sched %.3f (128) / %.3f (64) ms, %.3g / %.3g node-updates/s' % (max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled'], d['model'][1]['node_updates_per_s_overlapped'], d['model'][0]['node_updates_per_s_overlapped']))"
rm -f $d/*/kt_kernel_trace.csv 2>/dev/null; true
