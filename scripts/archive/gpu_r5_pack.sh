#!/bin/bash
# C5 at W = 8 virtual ranks: k_list_pack shapes (build/ablate/lib_<v>.so: 16 tiles per block; 16 tiles
# as 2 per wave; 8 / 16 payload slots in flight) against the product's (8 tiles, 4 slots), same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_pack}; mkdir -p $O
model() {  # model <tag> <W> <env...>
  local t=$1 W=$2; shift 2
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank max %.3f ms' % max(d['rank_compute_ms']), {k[:24]: round(sum(v)/len(v),3) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'])
for m in d['model']: print('   %g GB/s: sched %.3f ms -> %.3g' % (m['link_gbps'], m['round_ms_as_scheduled'], m['node_updates_per_s_overlapped']))"
}
model prod 8 GP_EXP=1 || exit 1
for v in lp16 lp16w2 pb8 pb16; do
  model $v 8 GP_EXP=1 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so || exit 1
done
model prod2 8 GP_EXP=1 || exit 1
