#!/bin/bash
# Round-6 end state, part C: modelled C5 rounds at W = 8 and W = 2 with the final code.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_final3}; mkdir -p $O
model() {  # model <tag> <n> <topo> <W>
  local t=$1 n=$2 topo=$3 w=$4
  local d=$O/vr_$t
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $n $topo push-sum $w 10 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d $n $topo push-sum $w 10 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank compute max %.3f ms, sched %.3f (128) / %.3f (64) ms' % (max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled']))
print('   per-slab kernels', {k: round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()}, 'global', {k: round(v,3) for k,v in d['global_kernel_ms'].items()})"
  rm -f $d/*/kt_kernel_trace.csv $d/kt_kernel_trace.csv 2>/dev/null; true
}
model c5w8 1000000000 Imp3D 8 && model c5w4 1000000000 Imp3D 4 && model c5w2 1000000000 Imp3D 2
