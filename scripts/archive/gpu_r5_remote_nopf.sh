#!/bin/bash
# The REMOTE round kernel with the sender prefetch compiled out (SNDPF = GP_SND_PF && !REMOTE):
# multi-rank parity, then the C5 W = 8 model.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_remote_nopf}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py > $O/pytest_multirank.log 2>&1 || { tail -30 $O/pytest_multirank.log; exit 1; }
tail -3 $O/pytest_multirank.log
d=$O/vr
GP_EXP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 8 20 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum 8 20 $O/model_c5w8.json > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('$O/model_c5w8.json'))
k=d['per_slab_kernel_ms']['k_ps_tile<3, true>']
print('round kernel %.3f ms/slab, rank max %.3f, sched %.3f / %.3f ms' % (sum(k)/len(k), max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled']))"
