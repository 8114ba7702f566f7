#!/bin/bash
# Eight exchange regions (and round-kernel launches) against four: virtual-rank parity of the
# experiments-build cases with GP_XREGIONS=8, then C5 at 2 / 4 / 8 virtual ranks, same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_reg8}; mkdir -p $O
GP_XREGIONS=8 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py -k "regions or tile" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
model() {  # model <tag> <W> <env...>
  local t=$1 w=$2; shift 2
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $w 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $w 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
k=[v for n,v in d['per_slab_kernel_ms'].items() if n.startswith('k_ps_tile')][0]
print('$t: round kernel %.3f ms/slab, rank max %.3f, sched %.3f (128) / %.3f (64) ms' % (sum(k)/len(k), max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled']))"
}
model w2_h8 2 GP_EXP=1 GP_XREGIONS=8 && model w2_h4 2 GP_EXP=1 GP_XREGIONS=4 && \
model w4_h8 4 GP_EXP=1 GP_XREGIONS=8 && model w4_h4 4 GP_EXP=1 GP_XREGIONS=4 && \
model w8_h8 8 GP_EXP=1 GP_XREGIONS=8 && model w8_h4 8 GP_EXP=1 GP_XREGIONS=4
