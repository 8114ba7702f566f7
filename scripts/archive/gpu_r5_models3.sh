#!/bin/bash
# C5 at 2 / 4 / 8 virtual ranks with the final round-5 code (lists in four regions, compacted halos,
# the tile kernel's sender prefetch) -- the DESIGN 7.1 end-state rows.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_models3}; mkdir -p $O
model() {  # model <tag> <W>
  local t=$1 W=$2
  local d=$O/vr_$t
  GP_EXP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank %.3f-%.3f ms' % (min(d['rank_compute_ms']), max(d['rank_compute_ms'])), {k[:22]: round(sum(v)/len(v),3) for k,v in d['per_slab_kernel_ms'].items()}, {k: round(v/$W,3) for k,v in d['global_kernel_ms'].items()})
for m in d['model']: print('   %g GB/s: exchange %.3f serial %.3f sched %.3f ms -> %.3g' % (m['link_gbps'], m['exchange_ms'], m['round_ms_serial'], m['round_ms_as_scheduled'], m['node_updates_per_s_overlapped']))"
}
model c5w8 8 && model c5w4 4 && model c5w2 2 && model c5w8b 8
