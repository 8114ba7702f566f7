#!/bin/bash
# C3 (Imp3D gossip, n = 1e8) at W = 2 / 4 / 8 as virtual ranks under a kernel trace: the per-rank round
# model (tools/mgpu_model.py), records into gpurun_out/r4_c3model.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c3model}
mkdir -p $O
for W in 2 4 8; do
  d=$O/vr_c3_w$W
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 100000000 Imp3D gossip $W 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python3 tools/mgpu_model.py model $d 100000000 Imp3D gossip $W 10 $O/model_c3_w$W.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/model_c3_w$W.json')); print($W, {k:round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'], [(m['link_gbps'], round(m['exchange_ms'],3), round(m['round_ms_serial'],3), '%.3g' % m['node_updates_per_s_serial']) for m in d['model']])"
done
