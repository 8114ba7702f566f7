#!/bin/bash
# Region-by-region rounds (gp_api.hip launch_round_regions) for Imp3D push-sum across ranks:
# multi-rank parity (virtual ranks, RCCL rank processes incl. C5 at 10^9 on 2 ranks), then the
# C5 model at 2 / 4 / 8 virtual ranks with (GP_RREGIONS=1) and without (=0), same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_rregions}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py tests/test_gpu_rccl_multiproc.py > $O/pytest_multirank.log 2>&1 || { tail -30 $O/pytest_multirank.log; exit 1; }
tail -3 $O/pytest_multirank.log
model() {  # model <tag> <W> <env...>
  local t=$1 w=$2; shift 2
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $w 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $w 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
k=[v for n,v in d['per_slab_kernel_ms'].items() if n.startswith('k_ps_tile')][0]
print('$t: round kernel %.3f ms/slab, rank max %.3f, sched %.3f (128) / %.3f (64) ms, regions %s' % (sum(k)/len(k), max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled'], d.get('round_regions')))"
}
model w2_r1 2 GP_EXP=1 GP_RREGIONS=1 && model w2_r0 2 GP_EXP=1 GP_RREGIONS=0 && \
model w4_r1 4 GP_EXP=1 GP_RREGIONS=1 && model w4_r0 4 GP_EXP=1 GP_RREGIONS=0 && \
model w8_r1 8 GP_EXP=1 GP_RREGIONS=1 && model w8_r0 8 GP_EXP=1 GP_RREGIONS=0
