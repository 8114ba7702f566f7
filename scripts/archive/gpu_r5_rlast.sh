#!/bin/bash
# Region rounds with the last region half the size of the others (GP_RLAST=1: its pack and
# transfer are the round's exposed tail) against equal regions (=0): parity of the forced-region
# virtual-rank cases, then C5 at 8 / 4 / 2 virtual ranks, same box, alternated at 8.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_rlast}; mkdir -p $O
GP_RLAST=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py -k "regions or timing" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
model() {  # model <tag> <W> <env...>
  local t=$1 w=$2; shift 2
  local d=$O/vr_$t
  env GP_EXP=1 "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $w 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $w 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank max %.3f, sched %.3f (128) / %.3f (64) ms, regions %s' % (max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled'], d.get('round_regions')))"
}
model w8_l1 8 GP_RLAST=1 && model w8_l0 8 GP_RLAST=0 && model w8_l1b 8 GP_RLAST=1 && model w8_l0b 8 GP_RLAST=0 && \
model w4_l1 4 GP_RLAST=1 && model w4_l0 4 GP_RLAST=0 && model w2_l1 2 GP_RLAST=1 && model w2_l0 2 GP_RLAST=0
