#!/bin/bash
# Multi-GPU model inputs after the two-region Imp3D push-sum exchange: C5 at W = 2, 4, 8 as virtual
# ranks under a kernel trace (tools/mgpu_model.py run / model), records into gpurun_out/r4_model2.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_model2}
mkdir -p $O
for W in 8 4 2; do
  d=$O/vr_c5_w$W
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  grep '^{' $d.log
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 10 $O/model_c5_w$W.json | tail -30 || exit 1
done
