#!/bin/bash
# Round-6 end state of the C5 kernels: C5 (1e9 Imp3D push-sum) to convergence on one GPU, and
# the multi-GPU round model at W = 2 / 4 / 8 (virtual ranks on one device, tools/mgpu_model.py).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_c5model}; mkdir -p $O
timeout -k 10 300 python3 tools/converge.py 1000000000 Imp3D push-sum 1 $O/c5_converge_1e9.json > $O/c5_converge.log 2>&1 || { tail -5 $O/c5_converge.log; exit 1; }
tail -2 $O/c5_converge.log
model() {  # model <tag> <W>
  local t=$1 w=$2
  local d=$O/vr_$t
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $w 10 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $w 10 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank compute max %.3f ms, sched %.3f (128) / %.3f (64) ms, %.3g / %.3g node-updates/s' % (max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled'], d['model'][1]['node_updates_per_s_overlapped'], d['model'][0]['node_updates_per_s_overlapped']))
print('   per-slab kernels', {k: round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()})"
  rm -f $d/*/kt_kernel_trace.csv $d/kt_kernel_trace.csv 2>/dev/null; true
}
model c5w8 8 && model c5w4 4 && model c5w2 2
