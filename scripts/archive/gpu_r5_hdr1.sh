#!/bin/bash
# REMOTE round kernel: a header word's mask and base in one 12-byte load (build/ablate/lib_hdr1.so,
# -DGP_HDR_ONE_LOAD=1) against two loads (the product), C5 at W = 8 virtual ranks, same box, alternated;
# variant parity first.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_hdr1}; mkdir -p $O
V=build/ablate/lib_hdr1.so
GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py -k "Imp3D and push" > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
model() {  # model <tag> <env...>
  local t=$1; shift
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 8 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum 8 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
k=d['per_slab_kernel_ms']['k_ps_tile<3, true>']
print('$t: round kernel %.3f ms/slab, rank max %.3f, sched %.3f / %.3f ms' % (sum(k)/len(k), max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled']))"
}
model prod GP_EXP=1 && model hdr1 GP_EXP=1 GOSSIP_HIP_LIB_EXPERIMENT=$V && model prod2 GP_EXP=1 && model hdr1b GP_EXP=1 GOSSIP_HIP_LIB_EXPERIMENT=$V
