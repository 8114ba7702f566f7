#!/bin/bash
# Region rounds with each region's pack on its own stream, beside the next region's round-kernel
# launch (GP_PSTREAM=1), against packs on the compute stream (=0): virtual-rank parity of the
# forced-region cases, then the C5 virtual-rank wall time per round (all W slabs on one GPU, so
# wall / W ~ one rank's compute with the overlap), alternated, W = 8 and 2.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_pstream}; mkdir -p $O
GP_PSTREAM=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py -k "regions or timing" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
wall() {  # wall <tag> <W> <env...>
  local t=$1 w=$2; shift 2
  env GP_EXP=1 "$@" timeout -k 10 300 python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $w 40 > $O/$t.log 2>&1 || { tail -20 $O/$t.log; return 1; }
  python3 -c "
import json
for l in open('$O/$t.log'):
    if l.startswith('{'): d=json.loads(l)
print('$t: wall %.3f ms/round, / W = %.3f' % (d['wall_ms_per_round_virtual'], d['wall_ms_per_round_virtual'] / $w))"
}
wall w8_p1 8 GP_PSTREAM=1 && wall w8_p0 8 GP_PSTREAM=0 && wall w8_p1b 8 GP_PSTREAM=1 && wall w8_p0b 8 GP_PSTREAM=0 && \
wall w2_p1 2 GP_PSTREAM=1 && wall w2_p0 2 GP_PSTREAM=0
