#!/bin/bash
# Multi-rank (virtual ranks) parity, then the multi-GPU model inputs for C5 / C4 at world 2/4/8.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_mr}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "parity: $(tail -1 $O/pytest.log)"
for cfg in ${CFGS:-"1000000000 Imp3D push-sum 8" "100000000 full push-sum 8"}; do :; done
IFS=';' read -ra CS <<< "${CFGS:-1000000000 Imp3D push-sum 8;1000000000 Imp3D push-sum 4;1000000000 Imp3D push-sum 2}"
for cfg in "${CS[@]}"; do
  set -- $cfg; d=$O/vr_$3_$2_$1_w$4
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $1 $2 $3 $4 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  grep '^{' $d.log
done
