#!/bin/bash
# Region rounds gated on slab size: multi-rank parity (virtual ranks incl. the forced-region cases,
# RCCL rank processes), the launcher tests, then the C5 W = 2 model (product build).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_rregions2}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py tests/test_gpu_rccl_multiproc.py tests/test_gpu_launcher.py --durations=12 > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -16 $O/pytest.log
d=$O/vr_w2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 2 20 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum 2 20 $O/model_c5w2.json > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('$O/model_c5w2.json'))
print('sched %.3f (128) / %.3f (64) ms, regions %s' % (d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled'], d.get('round_regions')))"
