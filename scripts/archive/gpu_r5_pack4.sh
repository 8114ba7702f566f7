#!/bin/bash
# C5 at W = 8 virtual ranks: k_list_pack with 4 tiles per 256-thread block (build/ablate/lib_lp4.so) against the
# product's 8, same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_pack4}; mkdir -p $O
model() {  # model <tag> <W> <env...>
  local t=$1 W=$2; shift 2
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('%-7s rank max %.3f ms  k_list_pack %.3f ms/slab  as scheduled 128 GB/s %.3f ms' % ('$t', max(d['rank_compute_ms']), d['global_kernel_ms']['k_list_pack']/8, d['model'][1]['round_ms_as_scheduled']))"
}
model prod 8 GP_EXP=1 && model lp4 8 GP_EXP=1 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_lp4.so && model prod2 8 GP_EXP=1 && model lp4b 8 GP_EXP=1 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_lp4.so
