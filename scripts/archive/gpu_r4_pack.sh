#!/bin/bash
# k_pack with batched buffer loads: virtual-rank and RCCL-process parity, then the W = 8 C5 model.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_pack}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl_multiproc.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
d=$O/vr_c5_w8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum 8 10 $O/model_c5_w8.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/model_c5_w8.json')); print(d['global_kernel_ms'], [m['round_ms_as_scheduled'] for m in d['model']])"
d=$O/vr_c3_w8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 100000000 Imp3D gossip 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
python3 tools/mgpu_model.py model $d 100000000 Imp3D gossip 8 10 $O/model_c3_w8.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/model_c3_w8.json')); print(d['global_kernel_ms'], [m['round_ms_as_scheduled'] for m in d['model']])"
