#!/bin/bash
# C5 at W = 8 virtual ranks: k_list_pack reading the round kernel's outbox (GP_OUTBOX=1; the REMOTE
# round kernel then stores (s, w) with plain stores so the outbox's re-read hits L2) against the
# (s, w) reads (same build, same box).  Parity of the outbox path first.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_outbox2}; mkdir -p $O
GP_OUTBOX=1 timeout -k 10 560 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py -k "Imp3D and push" > $O/multirank.log 2>&1 || { tail -30 $O/multirank.log; exit 1; }
tail -1 $O/multirank.log
model() {  # model <tag> <W> <env...>
  local t=$1 W=$2; shift 2
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank max %.3f ms' % max(d['rank_compute_ms']), {k[:24]: round(sum(v)/len(v),3) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'], d['pipelined_halves'])
for m in d['model']: print('   %g GB/s: sched %.3f ms -> %.3g' % (m['link_gbps'], m['round_ms_as_scheduled'], m['node_updates_per_s_overlapped']))"
}
model c5w8_sw 8 GP_EXP=1 && model c5w8_outbox 8 GP_EXP=1 GP_OUTBOX=1 && model c5w8_sw2 8 GP_EXP=1 || exit 1
