#!/bin/bash
# C4 (full push-sum, n = 1e8) at W = 8 virtual ranks: coarse bins at the rule vs one size smaller
# (GP_FB_S1D=-1, experiments build) -- per-rank round model from kernel traces, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4multi}
mkdir -p $O
for v in d0 m1; do
  if [ $v = m1 ]; then export GP_EXP=1 GP_FB_S1D=-1; else export GP_EXP=1; unset GP_FB_S1D; fi
  d=$O/vr_c4_w8_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 100000000 full push-sum 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python3 tools/mgpu_model.py model $d 100000000 full push-sum 8 10 $O/model_c4_w8_$v.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/model_c4_w8_$v.json')); print('$v', {k:round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'], [(m['link_gbps'], round(m['round_ms_as_scheduled'],3)) for m in d['model']])"
done
