#!/bin/bash
# End-state C5 model (product build: region rounds; eight regions at W = 2) at 2 / 4 / 8 virtual
# ranks, and the one-GPU bench on the same box for reference.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_models4}; mkdir -p $O
model() {  # model <tag> <W>
  local t=$1 w=$2
  local d=$O/vr_$t
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $w 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $w 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
k=[v for n,v in d['per_slab_kernel_ms'].items() if n.startswith('k_ps_tile')][0]
print('$t: round kernel %.3f ms/slab, rank max %.3f, sched %.3f (128) / %.3f (64) ms, %.3g / %.3g node-updates/s' % (sum(k)/len(k), max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled'], d['model'][1]['node_updates_per_s_overlapped'], d['model'][0]['node_updates_per_s_overlapped']))"
}
model c5w2 2 && model c5w4 4 && model c5w8 8 && \
timeout -k 10 300 python3 bench.py --no-cpu --no-traffic --steps 20 --warmup 3 > $O/bench1.json 2> $O/bench1.err && python3 -c "import json; d=json.load(open('$O/bench1.json')); print('one GPU: %.2f ms, %.3g' % (d['ms_per_step'], d['value']))"
