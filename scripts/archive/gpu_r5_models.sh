#!/bin/bash
# Round-5 per-rank models not yet recorded: C4 (full push-sum, P = 1e8) at 2 / 4 / 8 virtual ranks and
# C3 (Imp3D gossip, P = 100 544 625) at 4 (tools/mgpu_model.py).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_models}; mkdir -p $O
model() {  # model <tag> <n> <topo> <alg> <W> <rounds>
  local t=$1 n=$2 topo=$3 alg=$4 W=$5 R=$6
  local d=$O/vr_$t
  GP_EXP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $n $topo $alg $W $R > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d $n $topo $alg $W $R $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank %.3f-%.3f ms' % (min(d['rank_compute_ms']), max(d['rank_compute_ms'])), {k[:22]: round(sum(v)/len(v),3) for k,v in d['per_slab_kernel_ms'].items()}, {k: round(v/$W,3) for k,v in d['global_kernel_ms'].items()})
for m in d['model']: print('   %g GB/s: exchange %.3f serial %.3f sched %.3f ms share %.2f' % (m['link_gbps'], m['exchange_ms'], m['round_ms_serial'], m['round_ms_as_scheduled'], m['exchange_share_serial']))"
}
model c4w2 100000000 full push-sum 2 20 && model c4w4 100000000 full push-sum 4 20 && model c4w8 100000000 full push-sum 8 20 && model c3w4 100000000 Imp3D gossip 4 20
